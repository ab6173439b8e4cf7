#!/bin/bash
# Round 6 closing session: smoke, C++ reference tests, the adapter harness
# and full GPU suite, the default bench line and its rocprofv3 kernel-trace
# summary, and every method on every BASELINE config (with PMC traffic).
# Every GPU step has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${R06_OUT:-r06_final}; mkdir -p $OUT
export TMPDIR=/tmp
# SWEEP_ONLY=1: only the method sweep below (a second call, same OUT)
if [ "${SWEEP_ONLY:-0}" != 1 ]; then
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for t in test_downsampler test_downsampler_odd_z; do
  timeout -k 10 120 tests/cpp/bin/$t > $OUT/$t.log 2>&1 || { tail -20 $OUT/$t.log; exit 1; }
  tail -1 $OUT/$t.log
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_headline.json'));r=d['roofline'];c=d['cpu_baseline'];e=d['e2e'];print(d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], r['traffic'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), c['kind'], c['value'], e['ms_per_frame'], e['c2_filesystem_sink']['ms_per_frame'], d['library'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats*"
[ "${METHODS:-1}" = 1 ] || { echo "== done (no method sweep)"; exit 0; }
fi
for w in 4096x4096_u16 4096x4096_f32 1024x1024x256_u16 2048x2048_u16 512x512_u8; do
  for m in decimate mean min max; do
    timeout -k 10 300 python bench.py --workload $w --method $m --steps 20 --warmup 5 --cpu-seconds 0 \
      --e2e-frames 0 > $OUT/m_${w}_$m.json 2> $OUT/m_${w}_$m.err || { tail -20 $OUT/m_${w}_$m.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/m_${w}_$m.json'));r=d['roofline'];print('$w', '$m', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/methods.log
  done
done
# config V at one volume per launch too (the step size
# against the kernel), every launch rotated into HBM as above
for m in decimate mean min max; do
  timeout -k 10 300 python bench.py --workload 1024x1024x256_u16 --batch 256 --method $m --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 > $OUT/v1_$m.json 2> $OUT/v1_$m.err || { tail -20 $OUT/v1_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v1_$m.json'));r=d['roofline'];print('V1', '$m', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), r['buffer_sets'], d['config']['check'])" | tee -a $OUT/methods.log
done
python scripts/current_table.py $OUT > $OUT/current_table.md; cat $OUT/current_table.md
echo "== done"
