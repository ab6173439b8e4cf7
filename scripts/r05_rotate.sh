#!/bin/bash
# Round 5: the BASELINE configs whose launches read less than 1 GiB (V, C2,
# C1b), timed with rotating buffer sets (bench --rotate-mib 1024, the
# default) against one buffer set (the line's one_buffer_set_* fields), and
# the volume Decimate load policy under rotation ($AQZ_VOLUME_NT).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_rotate; mkdir -p $OUT
export TMPDIR=/tmp
run() { # name, extra env, bench args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];b=r.get('buffer_rotation') or {};c=r.get('same_mix_ceiling') or {};print('$n', r['buffer_sets'], r['avg_launch_us'], r['frac'], c.get('frac_of_ceiling'), c.get('GBps'), b.get('one_buffer_set_avg_launch_us'), b.get('one_buffer_set_frac'), d['config']['check'])" | tee -a $OUT/summary.log
}
for nt in 1 0; do
  run vdec_nt$nt AQZ_VOLUME_NT=$nt python bench.py --workload 1024x1024x256_u16 --method decimate --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc
done
for w in 1024x1024x256_u16 2048x2048_u16 512x512_u8; do
  for m in decimate mean min max; do
    run ${w}_$m AQZ_X=0 python bench.py --workload $w --method $m --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0
  done
done
echo "== done"
