#!/bin/bash
# Round 4, VERDICT r3 item 4: camera-format frames (rows that split 64-B
# bursts / 128-B lines), row-major and chunk-tiled levels, with PMC read and
# write traffic; then the pitch-matched probe (tools/pitch_probe.py) on the
# same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_shapes; mkdir -p $OUT
export TMPDIR=/tmp
for sh in 3000x3000 2600x2600 5472x3648 2000x2000 6000x4000 4096x4096; do
  for k in s t; do
    extra=""; [ $k = t ] && extra="--tiled"
    timeout -k 10 300 python bench.py --shape $sh $extra --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 \
      > $OUT/${k}_$sh.json 2> $OUT/${k}_$sh.err || { tail -20 $OUT/${k}_$sh.err; exit 1; }
    python -c "
import json
d=json.load(open('$OUT/${k}_$sh.json'));r=d['roofline'];t=r.get('traffic_detail') or {}
a=r['alg_bytes_per_launch']; rd=r.get('alg_read_bytes_per_launch')
print('$sh', 'tiled' if '$k'=='t' else 'rowmajor', r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/a,4), t.get('read_bytes'), t.get('write_bytes'), a, d['config'].get('batch_path'))" | tee -a $OUT/shapes.log
  done
done
timeout -k 10 300 python tools/pitch_probe.py --json $OUT/pitch_probe.jsonl > $OUT/pitch_probe.log 2>&1 || { tail -5 $OUT/pitch_probe.log; exit 1; }
cat $OUT/pitch_probe.log
echo "== done"
