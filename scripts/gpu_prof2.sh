set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o run --output-format csv -- python3 $R/bench.py --docs 100000 --steps 2 --warmup 1 --batch 64 > $R/gpurun_out/prof2.log 2>&1 || exit 1
