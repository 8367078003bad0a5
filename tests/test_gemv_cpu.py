"""CPU reference of the decode GEMV (ops.gemv_decode off the GPU): the four modes agree with the
unfused reference ops they replace on the GPU (rmsnorm -> linear -> residual add / SwiGLU /
rope_kv_), so the GPU kernel tests (tests/test_gemv_gpu.py) and this contract describe one op."""
import torch

from llm_kubernetes_minikube_sharp4dev_amd import ops
from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref


def _w(n, k, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, k, generator=g) * 0.05).to(torch.bfloat16)


def test_gemv_modes_match_unfused_reference():
    torch.manual_seed(0)
    K = 512
    x = torch.randn(2, K).to(torch.bfloat16)
    g = (torch.rand(K) + 0.5).to(torch.bfloat16)
    w = _w(256, K, 1)
    xn = ref.rmsnorm(x, g, 1e-5)
    # mode 0 with the norm prologue
    y = ops.gemv_decode(0, x, w, g, 1e-5)
    assert torch.equal(y, (xn.float() @ w.float().t()).to(torch.bfloat16))
    # mode 1: residual add in place
    res = torch.randn(2, 256).to(torch.bfloat16)
    want = ((x.float() @ w.float().t().float()).to(torch.bfloat16).float() + res.float()).to(torch.bfloat16)
    out = ops.gemv_decode(1, x, _w(256, K, 1), res=res)
    assert out is res and torch.equal(res, want)
    # mode 2: SwiGLU over [Wg; Wu]
    a = ops.gemv_decode(2, x, w, g, 1e-5)
    lin = (xn.float() @ w.float().t()).to(torch.bfloat16)
    assert a.shape == (2, 128)
    torch.testing.assert_close(a.float(), ref.silu_mul(lin).float(), atol=1e-2, rtol=1e-2)


def test_gemv_qkv_mode_writes_rotated_cache():
    Hq, Hkv, D, BS, K = 4, 2, 32, 16, 512
    N = (Hq + 2 * Hkv) * D
    x = torch.randn(1, K).to(torch.bfloat16)
    g = torch.ones(K, dtype=torch.bfloat16)
    w = _w(N, K, 3)
    cs = ops.rope_cos_sin(256, D, 10000.0)
    pos = torch.tensor([17], dtype=torch.int32)
    slots = torch.tensor([BS + 5], dtype=torch.int32)
    kc = torch.zeros(4, Hkv, BS, D, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    qkv = ops.gemv_decode(3, x, w, g, 1e-5, positions=pos, cos_sin=cs, Hq=Hq, Hkv=Hkv, D=D, k_cache=kc,
                          v_cache=vc, slots=slots, neox=True)
    lin = (ref.rmsnorm(x, g, 1e-5).float() @ w.float().t()).to(torch.bfloat16)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    want = ref.rope_kv_(lin.clone(), pos, cs, Hq, Hkv, D, kc2, vc2, slots, True, False)
    assert torch.equal(qkv, want)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    assert kc[1, :, 5].abs().sum() > 0 and kc[0].abs().sum() == 0
