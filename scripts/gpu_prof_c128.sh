set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --mode batch --batch 128 --steps 3 > gpurun_out/bench_b128_v4.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --mode batch --batch 64 --steps 3 > gpurun_out/bench_b64_v4.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c128 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/prof_c128.log 2>&1 || exit 3
