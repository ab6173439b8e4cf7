#!/bin/bash
# Round-2: f32 8-wave bands with 85 KiB of LDS (above the 64 KiB default),
# against the 64 KiB cap (direct stores); full GPU suite first.  r02m/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
  for w in "--workload 4096x4096_f32" ""; do
    for e in "AQZ_BAND_LDS_CAP=65536" "X=0" "AQZ_BAND_ALIGNED=0"; do
      env $e timeout -k 10 120 python bench.py $w --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$w', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/f32band_ab.log
    done
  done
done
echo "== done"
