set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "decode or cascade or engine" > gpurun_out/pytest_sp.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_sp.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_agent.sh
grep -E "decode_reduce|paged_decode|rmsnorm_kernel|rope_kv" gpurun_out/prof_agent_summary.md | head -8
