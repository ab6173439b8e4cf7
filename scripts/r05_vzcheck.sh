#!/bin/bash
# Round 5: the final library after the volume Decimate unit-order rule: the
# full GPU suite, smoke, and config V Decimate at 1 and 4 volumes per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_vzcheck; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for b in 256 1024; do
  timeout -k 10 200 python bench.py --workload 1024x1024x256_u16 --method decimate --batch $b --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 > $OUT/v_$b.json 2> $OUT/v_$b.err || { tail -20 $OUT/v_$b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v_$b.json'));r=d['roofline'];print('planes $b', r['buffer_sets'], r['avg_launch_us'], r['frac'], (r.get('same_mix_ceiling') or {}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'], d['library'])" | tee -a $OUT/v.log
done
echo "== done"
