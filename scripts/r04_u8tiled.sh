#!/bin/bash
# u8 camera frames, chunk 128: row-major against chunk-tiled, and the
# kernel-trace summary of the tiled batch.
set -e
out=gpurun_out/r04_u8tiled
mkdir -p $out
: > $out/ab.log
run() {  # shape extra-args
  timeout -k 10 120 python bench.py --workload 512x512_u8 --shape $1 $2 --steps 20 \
    --warmup 3 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $out/run.json
  python -c "import json;d=json.loads(open('$out/run.json').read().strip().splitlines()[-1]);c=d['config'];print('$1 $2', d['roofline']['avg_launch_us'], d['roofline']['frac'], c['batch_path'], c['launches_per_step'], c['frames_per_step_per_gpu'], c['levels'])" >> $out/ab.log
}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o u8 -- \
  python $GRAFT_REPO_ROOT/bench.py --workload 512x512_u8 --shape 2600x2600 --tiled --steps 10 \
  --warmup 2 --no-pmc --cpu-seconds 0 --e2e-frames 0 --no-check > $GRAFT_REPO_ROOT/$out/prof.log 2>&1
