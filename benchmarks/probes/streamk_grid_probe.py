import os, sys, statistics, torch, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from llm_kubernetes_minikube_sharp4dev_amd import ops
lib = ops.lib()
print("cus", torch.cuda.get_device_properties(0).multi_processor_count)
for M, N, K in ((2816, 4096, 4096), (3328, 4096, 14336), (4352, 4096, 4096)):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16); w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    res = {}
    for mode in (0, 1):
        lib.gemm_streamk(mode)
        for _ in range(3): lib.gemm(x, w, None, 0, 256, None, 2)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10): lib.gemm(x, w, None, 0, 256, None, 2)
        b.record(); torch.cuda.synchronize()
        res[mode] = a.elapsed_time(b) * 100
    print(json.dumps({"grid": os.environ.get("LK_GEMM_SK_GRID"), "M": M, "N": N, "K": K, "plain_us": round(res[0], 1), "sk_us": round(res[1], 1), "err": lib.gemm_streamk(-1)}), flush=True)
