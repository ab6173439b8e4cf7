#!/bin/bash
# Bit shuffle for 2-, 4- and 8-byte types: the 32x32 word transpose against
# the per-byte gather form ($AQZ_BITSHUFFLE_BYTES=1): codec parity both ways,
# then streamed time against a same-size D2D copy, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/bswords; mkdir -p $OUT
for by in 0 1; do
  AQZ_BITSHUFFLE_BYTES=$by timeout -k 10 300 python -u -m pytest tests/test_gpu_codecs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_codecs_b$by.log 2>&1 || { tail -30 $OUT/pytest_codecs_b$by.log; exit 1; }
  tail -1 $OUT/pytest_codecs_b$by.log
done
for rep in 1 2 3; do for by in 0 1; do
  echo "bytes=$by" >> $OUT/bitshuffle_ts.log
  AQZ_BITSHUFFLE_BYTES=$by timeout -k 10 200 python tools/bitshuffle_ts.py >> $OUT/bitshuffle_ts.log 2>&1 || { tail -20 $OUT/bitshuffle_ts.log; exit 1; }
done; done
grep -v amdgpu.ids $OUT/bitshuffle_ts.log
B="--cpu-seconds 0 --e2e-frames 4 --no-pmc --no-check --steps 5 --warmup 2"
for rep in 1 2; do for w in 4096x4096_u16 4096x4096_f32; do for by in 0 1; do
  AQZ_BITSHUFFLE_BYTES=$by timeout -k 10 300 python bench.py $B --workload $w > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/b.json'));s=d['e2e']['secondary_kernels']
b=s['blosc_bitshuffle'];c=s['d2d_copy_same_bytes']
print('bytes=$by $w bitshuffle',b['stream_us_per_frame'],b['avg_launch_us'],'copy',c['stream_us_per_frame'],'ratio',round(c['stream_us_per_frame']/b['stream_us_per_frame'],3))" | tee -a $OUT/bench_ab.log
done; done; done
echo "== done"
