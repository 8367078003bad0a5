set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py --model llama-3-70b --batch 64 --steps 2 --docs 1000000 > gpurun_out/wl_70b_1m.log 2>&1 || { tail gpurun_out/wl_70b_1m.log; exit 2; }
grep '"metric"' gpurun_out/wl_70b_1m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['config']['step_mix_rank0']; m.pop('host_breakdown'); print('70b-1m', d['value'], d['unit'], d['p50_latency_ms'], d['config']['corpus_chunks'], d['config']['index_build_s'], d['config']['stage_means_s'], json.dumps(m))"
