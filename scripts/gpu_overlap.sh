set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/ov_test.log 2>&1; rc=$?; tail -2 gpurun_out/ov_test.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1; do
LK_OVERLAP_ATTN=$v timeout -k 10 400 python bench.py --steps 3 > gpurun_out/ov_$v.log 2>&1 || exit 2
grep '"metric"' gpurun_out/ov_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap=$v', d['value'], d['p50_latency_ms'], d['config']['step_mix_rank0'])"
done
