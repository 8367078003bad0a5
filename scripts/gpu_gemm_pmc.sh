# PMC passes (one counter set per run) of the hand-written GEMM and hipBLASLt on one shape.
#   SHAPE="--M 4096 --N 4096 --K 14336" bash scripts/gpu_gemm_pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
SHAPE=${SHAPE:-"--M 4096 --N 4096 --K 14336"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
for impl in ours lib; do
  timeout -k 5 120 python benchmarks/gemm_one.py $SHAPE --impl $impl > gpurun_out/pmc/plain_$impl.log 2>&1 || exit 3
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc/${impl}_p$i -o run --output-format csv -- python3 benchmarks/gemm_one.py $SHAPE --impl $impl --iters 10 > gpurun_out/pmc/${impl}_p$i.log 2>&1 || { tail -5 gpurun_out/pmc/${impl}_p$i.log; exit 4; }
  done
done
cat gpurun_out/pmc/plain_*.log
