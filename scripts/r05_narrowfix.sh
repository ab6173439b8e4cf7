#!/bin/bash
# Round 5: 16-byte tiles only where every level row is whole bursts
# (W * b % 1024 == 0).  The whole GPU suite, then the f32 camera frames with
# counters (f32 5472x3648 had taken the narrow tile on its aligned level 0),
# and F 4096^2 f32, which must keep the narrow tile.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${R05_OUT:-r05_narrowfix}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
R05_OUT=${R05_OUT:-r05_narrowfix} WLS=4096x4096_f32 bash scripts/r05_shapes.sh || exit 1
for m in mean max decimate; do
  timeout -k 10 300 python bench.py --workload 4096x4096_f32 --method $m --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 > $OUT/f_$m.json 2> $OUT/f_$m.err || { tail -20 $OUT/f_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/f_$m.json'));r=d['roofline'];print('F', '$m', r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/f.log
done
echo "== done"
