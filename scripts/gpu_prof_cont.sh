set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/kernel_bench.py gemm_sweep --md gpurun_out/gemm_sweep.md > gpurun_out/gemm_sweep.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c256 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --batch 256 > $R/gpurun_out/prof_c256.log 2>&1 || exit 2
