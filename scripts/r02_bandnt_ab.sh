#!/bin/bash
# Round-2 A/B: the band kernel's loads follow the launcher's cache policy
# (non-temporal unless rows split 128-B lines) instead of always nt
# ($AQZ_LOAD_NT=1 = the old behaviour); misaligned <= 4-tile bands.  r02r/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02r; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
  for w in "" "--shape 2000x2000" "--shape 1500x1500" "--shape 1000x1000" "--shape 2040x2048"; do
    for e in "AQZ_LOAD_NT=1" "X=0" "AQZ_BAND_ALIGNED=0"; do
      [ -n "$w" ] && [ "$e" = "AQZ_BAND_ALIGNED=0" ] && continue
      env $e timeout -k 10 120 python bench.py $w --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$w', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/bandnt_ab.log
    done
  done
done
echo "== done"
