# PMC passes over the two attention kernels at their serving shapes (flash prefill on the
# in-situ chunk, paged decode at B128 x 1000 keys): MFMA busy / clock / waits, LDS behaviour,
# HBM bytes.  One counter set per rocprofv3 run (slot limits: MI355X_MICROARCH.md), each under
# its own timeout; stop at the first failure.  Summaries: scripts/gemm_pmc_table.py, pmc_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/attn_pmc
cd /tmp && export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SALU"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
run() {  # tag counters command...
  tag=$1; ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -d $R/gpurun_out/attn_pmc/$tag -o run --output-format csv -- "$@" \
    > $R/gpurun_out/attn_pmc/$tag.log 2>&1 || { tail -5 $R/gpurun_out/attn_pmc/$tag.log; exit 2; }
}
for p in 1 2 3; do
  eval ctr=\$P$p
  run flash_chunk_p$p "$ctr" python3 $R/benchmarks/flash_one.py --shape chunk --iters 40 || exit 2
  run decode_b128_p$p "$ctr" python3 $R/benchmarks/decode_one.py --B 128 --ctx 1000 --iters 40 || exit 2
done
cd $R
python3 scripts/gemm_pmc_table.py gpurun_out/attn_pmc/flash_chunk_p1 gpurun_out/attn_pmc/decode_b128_p1 \
  --md gpurun_out/attn_pmc/clock_busy.md
{ python3 scripts/pmc_summary.py gpurun_out/attn_pmc/flash_chunk_p2 gpurun_out/attn_pmc/flash_chunk_p3 --kernel flash_prefill
  python3 scripts/pmc_summary.py gpurun_out/attn_pmc/decode_b128_p2 gpurun_out/attn_pmc/decode_b128_p3 --kernel paged_decode
} > gpurun_out/attn_pmc/counters.txt
cat gpurun_out/attn_pmc/counters.txt
find gpurun_out/attn_pmc -name "*.csv" -size +20M -delete
