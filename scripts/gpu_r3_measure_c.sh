# round 3 measurements, part C: decode-regime GEMM routing data (cold weights), then the HTTP
# split server vs one-process server vs in-process at 128 sessions
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u benchmarks/decode_route.py --json gpurun_out/r3c/decode_route.json > gpurun_out/r3c/decode_route.log 2>&1 || { tail gpurun_out/r3c/decode_route.log; exit 1; }
python -c "
import json
for r in json.load(open('gpurun_out/r3c/decode_route.json'))['rows']:
    print(r['shape'], r['M'], r.get('ws_us'), r.get('gemm_us'), r['hipblaslt_us'], r['policy'], r['policy_vs_hipblaslt'], r['policy_vs_best_own'])
"
bash scripts/gpu_http_split.sh
