# PMC pass of the flash-prefill kernel variants (causal B8 L4096): MFMA busy, waits, LDS
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_flash
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS"
for cfg in "8 0" "8 1" "4 0"; do
  set -- $cfg
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    LK_PREFILL_WAVES=$1 LK_PREFILL_PIPE=$2 timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_flash/w$1p$2_p$i -o run --output-format csv -- python3 benchmarks/flash_one.py --iters 5 > gpurun_out/pmc_flash/w$1p$2_p$i.log 2>&1 || { tail -5 gpurun_out/pmc_flash/w$1p$2_p$i.log; exit 4; }
  done
done
echo done
