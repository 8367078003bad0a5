"""Context-parallel attention on the flash kernel (models/attention.py cp_local_partials): each
CP "rank" holds one contiguous shard of every sequence's keys in its paged cache; its partials
come from the flash kernel in partial mode (prefill rows causal with the mask shifted by the
shard's first key position via ``q_past``, decode rows as one-query sequences), converted to
(o, lse) and LSE-merged.  The merge over 1, 2 and 3 shards (some empty) must match the fp32
reference of the unsharded problem.  The all-gather between ranks is the only part not run
here (the gloo CPU test covers it: tests/test_parallel_cpu.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SEQS = [("prefill", 300, 70), ("prefill", 130, 130), ("prefill", 600, 33), ("decode", 500, 1), ("decode", 20, 1),
        ("decode", 129, 1)]  # (kind, ctx, q)
HQ, HKV, D, BS = 8, 2, 128, 16


def _problem(C, rank, dev):
    from llm_kubernetes_minikube_sharp4dev_amd.models.attention import AttnMeta

    g = torch.Generator().manual_seed(11)
    keys = [(torch.randn(n, HKV, D, generator=g).to(torch.bfloat16), torch.randn(n, HKV, D, generator=g).to(torch.bfloat16))
            for _, n, _ in SEQS]
    q = [torch.randn(ql, HQ, D, generator=g).to(torch.bfloat16) for _, _, ql in SEQS]
    kc = torch.zeros(256, HKV, BS, D, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    nxt, tables, lens, starts = 0, [], [], []
    for (k, v), (_, n, _) in zip(keys, SEQS):
        per = -(-n // C)
        a, b = min(n, rank * per), min(n, (rank + 1) * per)
        nb = max(1, -(-(b - a) // BS))
        blocks = list(range(nxt, nxt + nb))
        nxt += nb
        for j in range(b - a):
            kc[blocks[j // BS], :, j % BS] = k[a + j]
            vc[blocks[j // BS], :, j % BS] = v[a + j]
        tables.append(blocks + [0] * (48 - nb))
        lens.append(b - a)
        starts.append(a)
    pre = [i for i, s in enumerate(SEQS) if s[0] == "prefill"]
    dec = [i for i, s in enumerate(SEQS) if s[0] == "decode"]
    qrows = torch.cat([q[i] for i in pre + dec])
    T = qrows.shape[0]
    qkv = torch.zeros(T, (HQ + 2 * HKV) * D, dtype=torch.bfloat16)
    qkv[:, : HQ * D] = qrows.reshape(T, -1)
    pos = []
    for i in pre:
        n, ql = SEQS[i][1], SEQS[i][2]
        pos += list(range(n - ql, n))
    pos += [SEQS[i][1] - 1 for i in dec]
    cu = [0]
    for i in pre:
        cu.append(cu[-1] + SEQS[i][2])
    i32 = dict(dtype=torch.int32, device=dev)
    meta = AttnMeta(positions=torch.tensor(pos, **i32), slots=torch.full((T,), -1, **i32),
                    num_prefill_tokens=cu[-1], num_prefill_seqs=len(pre), num_decode=len(dec),
                    cu_q=torch.tensor(cu, **i32), ctx_lens_p=torch.tensor([lens[i] for i in pre], **i32),
                    block_tables_p=torch.tensor([tables[i] for i in pre], **i32),
                    q_lens_cpu=[SEQS[i][2] for i in pre], ctx_lens_cpu=[lens[i] for i in pre],
                    block_tables_d=torch.tensor([tables[i] for i in dec], **i32),
                    ctx_lens_d=torch.tensor([lens[i] for i in dec], **i32),
                    cp_key_start_p=[starts[i] for i in pre], cp_key_start_d=[starts[i] for i in dec])
    return qkv.to(dev), kc.to(dev), vc.to(dev), meta


@pytest.mark.parametrize("C", [1, 2, 3])
def test_cp_partials_on_the_flash_kernel_merge_to_the_reference(C):
    from llm_kubernetes_minikube_sharp4dev_amd.models.attention import cp_local_partials, merge_partials

    scale = D ** -0.5
    qkv, kc, vc, meta = _problem(1, 0, "cpu")
    qkv, kc, vc = qkv.float(), kc.float(), vc.float()
    o_ref, l_ref = cp_local_partials(qkv, kc, vc, meta, HQ, HKV, D, scale)  # fp32, unsharded
    os_, ls = [], []
    for r in range(C):
        qkv, kc, vc, meta = _problem(C, r, "cuda")
        o, lse = cp_local_partials(qkv, kc, vc, meta, HQ, HKV, D, scale)
        os_.append(o)
        ls.append(lse)
    got = merge_partials(torch.stack(os_), torch.stack(ls)).cpu()
    torch.testing.assert_close(got, o_ref, atol=2e-2, rtol=2e-2)
    if C == 1:
        lse = ls[0].cpu()
        torch.testing.assert_close(lse, l_ref, atol=1e-2, rtol=1e-3)
