set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/wl_$tag.log 2>&1 || { tail -20 gpurun_out/wl_$tag.log; exit 1; }; grep '"metric"' gpurun_out/wl_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['metric'], d['value'], d['p50_latency_ms'], c['seq_len'], c['http_status_counts_rank0'], c['step_mix_rank0'])"; }
run rag_default
run agent --workload agent
run mixed --workload mixed
run rag70b --model llama-3-70b --batch 64 --steps 2
