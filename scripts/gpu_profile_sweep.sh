set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --docs 20000 --steps 1 --warmup 1 --batch 32 > $R/gpurun_out/prof1.log 2>&1 || exit 1
cd $R
for B in 64 128; do
  timeout -k 10 600 python3 bench.py --docs 100000 --steps 3 --warmup 1 --batch $B > gpurun_out/bench_b$B.log 2>&1 || exit 2
done
