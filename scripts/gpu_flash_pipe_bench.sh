set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fpipe
for r in 1 2; do
  for cfg in "4 0" "4 1" "8 0" "8 1"; do
    set -- $cfg
    LK_PREFILL_WAVES=$1 LK_PREFILL_PIPE=$2 timeout -k 10 200 python benchmarks/kernel_bench.py prefill encoder > gpurun_out/fpipe/w$1p$2_r$r.log 2>&1 || { tail gpurun_out/fpipe/w$1p$2_r$r.log; exit 2; }
    echo "round $r waves $1 pipe $2"; grep case gpurun_out/fpipe/w$1p$2_r$r.log
  done
done
