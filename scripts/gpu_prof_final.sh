set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_v6 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/prof_v6.log 2>&1 || exit 1
grep '"metric"' $R/gpurun_out/prof_v6.log | cut -c1-200
