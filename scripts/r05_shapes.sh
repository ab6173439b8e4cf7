#!/bin/bash
# Round 5: camera-format frames on the final library, row-major and
# chunk-tiled, u16 and f32, with PMC reads and writes each against their
# algorithmic bytes (look further only where a counter shows
# more than 3% excess).  Columns: label, us per launch, of spec, of
# ceiling, reads / algorithmic, writes / algorithmic.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${R05_OUT:-r05_shapes}; mkdir -p $OUT
export TMPDIR=/tmp
SHAPES=${SHAPES:-"3000x3000 2600x2600 5472x3648 2000x2000 6000x4000 4100x4100"}
WLS=${WLS:-"4096x4096_u16 4096x4096_f32"}
for w in $WLS; do
  for s in $SHAPES; do
    for lay in rowmajor tiled; do
      a=""; [ $lay = tiled ] && a="--tiled"
      tag=${w##*_}_${s}_$lay
      env ${ENVS:-AQZ_UNUSED=0} timeout -k 10 300 python bench.py --workload $w --shape $s $a --steps 20 --warmup 5 \
        --cpu-seconds 0 --e2e-frames 0 > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
      python -c "
import json;d=json.load(open('$OUT/$tag.json'));r=d['roofline'];t=r.get('traffic_detail') or {}
ar=r['alg_read_bytes_per_launch'];aw=r['alg_bytes_per_launch']-ar
print('$tag', r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'),
      t and round(t['read_bytes']/ar,4), t and round(t['write_bytes']/aw,4), d['config']['check'])" | tee -a $OUT/shapes.log
    done
  done
done
echo "== done"
