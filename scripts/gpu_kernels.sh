set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -k "decode" > gpurun_out/kt_decode.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/kernel_bench.py --md gpurun_out/kernels.md > gpurun_out/kernels.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --docs 100000 --steps 3 --warmup 1 --batch 64 > gpurun_out/bench_b64_v1.log 2>&1 || exit 3
