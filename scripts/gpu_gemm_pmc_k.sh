# PMC pass of the prefill GEMM at two K (same M, N: 7 waves of tiles) to split the per-tile
# fixed cost from the K-proportional work: counters per dispatch, K 1024 vs 4096
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmck
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"
for K in 1024 4096; do
  timeout -k 5 120 python benchmarks/gemm_one.py --M 4096 --N 28672 --K $K --iters 20 > gpurun_out/pmck/plain_$K.log 2>&1 || exit 3
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmck/k${K}_p$i -o run --output-format csv -- python3 benchmarks/gemm_one.py --M 4096 --N 28672 --K $K --iters 6 > gpurun_out/pmck/k${K}_p$i.log 2>&1 || { tail -5 gpurun_out/pmck/k${K}_p$i.log; exit 4; }
  done
done
cat gpurun_out/pmck/plain_*.log
