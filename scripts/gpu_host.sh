set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for mode in "" "--unconstrained"; do
timeout -k 10 400 python bench.py $mode > gpurun_out/bench_host.log 2>&1 || exit 1
grep '"metric"' gpurun_out/bench_host.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; print('$mode', d['value'], d['ms_per_step'], m['host_breakdown'], m['decode_only_s'], m['mixed_s'])"
done
