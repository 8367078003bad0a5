# TP prefill overlap evidence: `bench.py --tp 2 --one-device` (2 ranks sharing the box's MI355X,
# IPC collectives) with each rank under its own rocprofv3 kernel trace; scripts/tp_overlap.py
# then reports, per rank, how much of every chunked all-reduce+norm kernel (comm stream) ran
# while a GEMM of the same process (compute stream) was running.  Output: gpurun_out/tp_overlap/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tp_overlap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 WORLD_SIZE=2 LK_TRACE_WINDOW=1 LK_ONE_DEVICE_HW_QUEUES=4
ARGS="--gpus 2 --tp 2 --one-device --docs 2000 --batch 32 --steps 2 --warmup 1 --max-new-tokens 16"
RANK=1 LOCAL_RANK=1 timeout -k 10 500 rocprofv3 --kernel-trace -d $O/r1 -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/r1.log 2>&1 &
P1=$!
RANK=0 LOCAL_RANK=0 timeout -k 10 500 rocprofv3 --kernel-trace -d $O/r0 -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/r0.log 2>&1
RC0=$?
wait $P1
RC1=$?
[ $RC0 -eq 0 ] && [ $RC1 -eq 0 ] || { tail -20 $O/r0.log; tail -20 $O/r1.log; exit 21; }
grep '"metric"' $O/r0.log | cut -c1-300
cd $R && for r in 0 1; do
  f=$(ls $O/r$r/*/run_kernel_trace.csv $O/r$r/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/tp_overlap.py $f > $O/overlap_r$r.md && gzip -c $f > $O/kernel_trace_r$r.csv.gz && rm -f $f
done
head -30 $O/overlap_r0.md
