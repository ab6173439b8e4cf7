#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
for wv in 1 2; do
AQZ_BITSHUFFLE_WAVES=$wv timeout -k 10 300 python -u -m pytest tests/test_gpu_codecs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_codecs_w$wv.log 2>&1 || { tail -30 $OUT/pytest_codecs_w$wv.log; exit 1; }
tail -1 $OUT/pytest_codecs_w$wv.log
done
B="--cpu-seconds 0 --e2e-frames 4 --no-pmc --no-check --steps 5 --warmup 2"
for rep in 1 2; do for w in 4096x4096_f32 4096x4096_u16; do for wv in 4 2 1; do
  AQZ_BITSHUFFLE_WAVES=$wv timeout -k 10 300 python bench.py $B --workload $w > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/b.json'));s=d['e2e']['secondary_kernels']
b=s['blosc_bitshuffle'];c=s['d2d_copy_same_bytes']
print('waves=$wv $w bitshuffle',b['stream_us_per_frame'],'copy',c['stream_us_per_frame'],'ratio',round(c['stream_us_per_frame']/b['stream_us_per_frame'],3))" | tee -a $OUT/bitshuffle_waves_ab.log
done; done; done
