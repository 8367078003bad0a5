# gemm4w loop ablations (timing only): 0 full, 2 no fragment reads, 3 no DMA, 4 neither; + gemm.hip s2, hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g4abl
cat > /tmp/abl.py <<'PY'
import sys, torch, statistics
sys.path.insert(0, ".")
from llm_kubernetes_minikube_sharp4dev_amd import ops
import torch.nn.functional as F
L = ops.lib()
for (M, N, K) in [(8192, 4096, 14336), (8192, 4096, 4096)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    fns = {f"4w_v{v}": (lambda v=v: L.gemm4w(x, w, None, 0, None, 1, v)) for v in (0, 6, 5, 7)}
    fns["8w_s2"] = lambda: L.gemm(x, w, None, 0, 256, None, 2, 1)
    fns["lib"] = lambda: F.linear(x, w)
    for f in fns.values():
        f()
    ts = {k: [] for k in fns}
    for _ in range(10):
        for k, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); f(); b.record(); b.synchronize()
            ts[k].append(a.elapsed_time(b) * 1e3)
    fl = 2.0 * M * N * K
    print(M, N, K, {k: (round(statistics.median(v), 1), round(fl / statistics.median(v) / 1e6)) for k, v in ts.items()}, flush=True)
PY
timeout -k 10 300 python /tmp/abl.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/g4abl/abl.log
