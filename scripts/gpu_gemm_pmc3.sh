# PMC passes of gemm.hip (schedule 2), gemm4w.hip and hipBLASLt on one shape.
#   SHAPE="--M 8192 --N 4096 --K 14336" bash scripts/gpu_gemm_pmc3.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
SHAPE=${SHAPE:-"--M 8192 --N 4096 --K 14336"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES"
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc3/counters.txt 2>&1 || true
for impl in ours 4w lib; do
  timeout -k 5 120 python benchmarks/gemm_one.py $SHAPE --impl $impl --variant 2 > gpurun_out/pmc3/plain_$impl.log 2>&1 || exit 3
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc3/${impl}_p$i -o run --output-format csv -- python3 benchmarks/gemm_one.py $SHAPE --impl $impl --variant 2 --iters 10 > gpurun_out/pmc3/${impl}_p$i.log 2>&1 || { tail -5 gpurun_out/pmc3/${impl}_p$i.log; exit 4; }
  done
done
cat gpurun_out/pmc3/plain_*.log
