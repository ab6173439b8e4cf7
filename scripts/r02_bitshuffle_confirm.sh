#!/bin/bash
# Bit shuffle defaults after the word transpose: codec parity, per-typesize
# streamed time, and the headline's secondary_kernels line.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/bsconfirm; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_codecs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_codecs.log 2>&1 || { tail -30 $OUT/pytest_codecs.log; exit 1; }
tail -1 $OUT/pytest_codecs.log
timeout -k 10 200 python tools/bitshuffle_ts.py > $OUT/bitshuffle_ts.log 2>&1 || { tail -20 $OUT/bitshuffle_ts.log; exit 1; }
grep -v amdgpu.ids $OUT/bitshuffle_ts.log
B="--cpu-seconds 0 --e2e-frames 4 --no-pmc --no-check --steps 5 --warmup 2"
for w in 4096x4096_u16 4096x4096_f32; do
  timeout -k 10 300 python bench.py $B --workload $w > $OUT/b_$w.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/b_$w.json'));s=d['e2e']['secondary_kernels']
b=s['blosc_bitshuffle'];c=s['d2d_copy_same_bytes']
print('$w bitshuffle',b['stream_us_per_frame'],b['avg_launch_us'],'copy',c['stream_us_per_frame'],'ratio',round(c['stream_us_per_frame']/b['stream_us_per_frame'],3))"
done
echo "== done"
