# Prefill GEMM vs hipBLASLt at the served M = 4096: un-profiled time, then one PMC pass per
# (shape, impl) with the kernel trace for durations -> effective clock and MFMA busy
# (scripts/gemm_pmc_table.py).  Each GPU step under its own timeout; stop at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pwr
SHAPES="qkv:6144:4096:none o:4096:4096:none gateup:28672:4096:swiglu down:4096:14336:none"
for s in $SHAPES; do
  IFS=: read name n k epi <<< "$s"
  for impl in prod lib; do
    timeout -k 10 120 python3 benchmarks/gemm_one.py --M 4096 --N $n --K $k --epi $epi --impl $impl --iters 100 \
      >> gpurun_out/pwr/timing.log 2>&1 || exit 1
  done
done
cat gpurun_out/pwr/timing.log
cd /tmp && export TMPDIR=/tmp
CTRS="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY"
DIRS=""
for s in $SHAPES; do
  IFS=: read name n k epi <<< "$s"
  for impl in prod lib; do
    d=$R/gpurun_out/pwr/${name}_${n}_${k}_4096_${impl}
    timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace -d $d -o run --output-format csv -- \
      python3 $R/benchmarks/gemm_one.py --M 4096 --N $n --K $k --epi $epi --impl $impl --iters 40 \
      > $d.log 2>&1 || { tail -5 $d.log; exit 2; }
    DIRS="$DIRS $d"
  done
done
cd $R && python3 scripts/gemm_pmc_table.py $DIRS --md gpurun_out/pwr/gemm_power.md
