# kernel trace of the headline bench -> where the device idles between kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/gap
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/gap/prof -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 > $R/gpurun_out/gap/prof.log 2>&1 || exit 1
cd $R && f=$(ls gpurun_out/gap/prof/*/run_kernel_trace.csv gpurun_out/gap/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/gap_context.py $f 4.0 100 > gpurun_out/gap/gaps.md && python3 scripts/gap_context.py $f 3.0 100 2.5 > gpurun_out/gap/gaps_mid.md && python3 scripts/gap_context.py $f 3.0 100 6.0 >> gpurun_out/gap/gaps_mid.md || exit 3
rm -rf gpurun_out/gap/prof
cat gpurun_out/gap/gaps_mid.md; grep -c . gpurun_out/gap/prof.log
