#!/bin/bash
# Bit shuffle for 4- and 8-byte types: DPP lane-group row stores against one
# lane per row piece ($AQZ_BITSHUFFLE_PAIR=0), codec parity both ways, then
# streamed time against a same-size D2D copy, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/bspair; mkdir -p $OUT
for pr in 1 0; do
  AQZ_BITSHUFFLE_PAIR=$pr timeout -k 10 300 python -u -m pytest tests/test_gpu_codecs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_codecs_p$pr.log 2>&1 || { tail -30 $OUT/pytest_codecs_p$pr.log; exit 1; }
  tail -1 $OUT/pytest_codecs_p$pr.log
done
B="--cpu-seconds 0 --e2e-frames 4 --no-pmc --no-check --steps 5 --warmup 2"
for rep in 1 2 3; do for pr in 1 0; do
  AQZ_BITSHUFFLE_PAIR=$pr timeout -k 10 300 python bench.py $B --workload 4096x4096_f32 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "
import json;d=json.load(open('$OUT/b.json'));s=d['e2e']['secondary_kernels']
b=s['blosc_bitshuffle'];c=s['d2d_copy_same_bytes']
print('pair=$pr f32 bitshuffle',b['stream_us_per_frame'],b['avg_launch_us'],'copy',c['stream_us_per_frame'],'ratio',round(c['stream_us_per_frame']/b['stream_us_per_frame'],3))" | tee -a $OUT/bitshuffle_pair_ab.log
done; done
for rep in 1 2; do for pr in 1 0; do
  echo "pair=$pr" | tee -a $OUT/bitshuffle_ts.log
  AQZ_BITSHUFFLE_PAIR=$pr timeout -k 10 200 python tools/bitshuffle_ts.py >> $OUT/bitshuffle_ts.log 2>&1 || { tail -20 $OUT/bitshuffle_ts.log; exit 1; }
done; done
cat $OUT/bitshuffle_ts.log
echo "== done"
