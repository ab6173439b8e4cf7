#!/bin/bash
# Round 4: after the units-per-wave rule — full GPU suite, every BASELINE
# config x method (with PMC traffic), and 512^2 u8 Decimate at 8 units per
# wave against the rule's 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_verify; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for w in 512x512_u8 4096x4096_u16 4096x4096_f32 1024x1024x256_u16 2048x2048_u16; do
  for m in decimate mean min max; do
    timeout -k 10 300 python bench.py --workload $w --method $m --steps 20 --warmup 5 --cpu-seconds 0 \
      --e2e-frames 0 > $OUT/m_${w}_$m.json 2> $OUT/m_${w}_$m.err || { tail -20 $OUT/m_${w}_$m.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/m_${w}_$m.json'));r=d['roofline'];print('$w', '$m', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/methods.log
  done
done
for u in 8 0; do
  AQZ_UNITS_PER_WAVE=$u timeout -k 10 300 python bench.py --workload 512x512_u8 --method decimate --steps 30 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('u8dec upw=$u', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'])" | tee -a $OUT/methods.log
done
echo "== done"
