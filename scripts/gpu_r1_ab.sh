# regression hunt: the round-1 tree (_r1/, git worktree of dbc0922, built in-tree) vs this tree,
# same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r1ab
run() {  # tag, dir, args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 500 python bench.py "$@" --json-out $GRAFT_REPO_ROOT/gpurun_out/r1ab/$tag.json > $GRAFT_REPO_ROOT/gpurun_out/r1ab/$tag.log 2>&1) || { echo "FAIL $tag"; tail -5 gpurun_out/r1ab/$tag.log; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r1ab/$tag.json')); c=d['config']; print('$tag', d['value'], 'p50', d['p50_latency_ms'], 'seq', c.get('seq_len'))"
}
run r1 _r1 && run r2 . && run r2_old_sched . --max-batched-tokens 4096 --admit-chunk 8 --admission inline --tokenizer benchmarks/data/bpe_runbooks_r1.json && run r1b _r1 && run r2b .
