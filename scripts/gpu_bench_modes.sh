set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --batch 128 > gpurun_out/bench_c128.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --batch 64 > gpurun_out/bench_c64.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --batch 128 --max-batched-tokens 4096 > gpurun_out/bench_c128_t4k.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch 256 > gpurun_out/bench_c256.log 2>&1 || exit 4
