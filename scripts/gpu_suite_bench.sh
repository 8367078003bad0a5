# GPU test suite, smoke, then the headline bench (default config) with its JSON
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
echo smoke-ok
timeout -k 10 500 python bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); c=d['config']; print(d['value'], d['p50_latency_ms'], c['seq_len'], c.get('chars_per_token'), c.get('prompt_chars'), c['stage_means_s'])"
