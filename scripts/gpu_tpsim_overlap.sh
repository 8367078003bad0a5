# 70B TP=8 rank-0 shard (--tp-sim 8): the TP prefill pipeline's compute cost, interleaved, twice:
# LK_TP_OVERLAP=1 (4 row chunks from 1024 rows), =0 (whole-step GEMMs), chunks 2 from 4096 rows.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/tpsim_ov
for i in 1 2; do
  for arm in on off c2; do
    case $arm in on) E="LK_TP_OVERLAP=1";; off) E="LK_TP_OVERLAP=0";; c2) E="LK_TP_OVERLAP_CHUNKS=2 LK_TP_OVERLAP_MIN_ROWS=4096";; esac
    env $E timeout -k 10 600 python bench.py --model llama-3-70b --tp-sim 8 --batch 64 --steps 8 --warmup 1 --json-out gpurun_out/tpsim_ov/${arm}_$i.json > gpurun_out/tpsim_ov/${arm}_$i.log 2>&1 || { tail gpurun_out/tpsim_ov/${arm}_$i.log; exit 94; }
    python -c "
import json; d=json.load(open('gpurun_out/tpsim_ov/${arm}_$i.json')); c=d['config']; m=c['step_mix_rank0']; e=c.get('collective_estimate') or {}
lf=e.get('latency_floor_plus_bytes',{}); up=e.get('upper',{})
print('$arm', d['value'], d['p50_latency_ms'], 'mixed ms', round(1e3*m['mixed_gpu_s']/max(1,m['mixed_steps']),2), 'dec ms', round(1e3*m['decode_only_gpu_s']/max(1,m['decode_only_steps']),2), 'exposed coll ms/step', lf.get('ms_per_step'), up.get('ms_per_step'), 'vs_elapsed', lf.get('vs_elapsed'), up.get('vs_elapsed'))"
  done
done
