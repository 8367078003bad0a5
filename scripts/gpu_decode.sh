set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -x -k "decode" > gpurun_out/kt_decode.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/kernel_bench.py decode prefill encoder knn --md gpurun_out/kernels_decode.md > gpurun_out/kernels_decode.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --docs 100000 --steps 3 --warmup 1 --batch 64 > gpurun_out/bench_b64_v3.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --docs 100000 --steps 3 --warmup 1 --batch 128 > gpurun_out/bench_b128_v3.log 2>&1 || exit 4
