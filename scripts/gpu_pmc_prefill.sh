set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 200 python benchmarks/kernel_bench.py prefill > gpurun_out/prefill_bench.log 2>&1 || exit 1
cat gpurun_out/prefill_bench.log | grep case
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_prefill -o run -- python3 $R/benchmarks/kernel_bench.py prefill_chunk > $R/gpurun_out/pmc_prefill.log 2>&1 || { tail -20 $R/gpurun_out/pmc_prefill.log; exit 2; }
ls $R/gpurun_out/pmc_prefill
