#!/bin/bash
# Round 6: the product with unmasked edge loads.  The new
# regression test (product and the divergent build over the new loads, under
# round 5's launch), the fuzz suite, the printf build on the old masked form
# (in-range edge chunks that load as all-zero bits), and the cost of the
# change: product vs the masked-load build on frames with right/bottom edges
# (f32 and u8, the types shard 0 holds), alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${R06_OUT:-r06_edgeab}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_divergent.py tests/test_gpu_fuzz.py -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
if [ -f tools/divergent/lib_divdbg.so ]; then
  env AQZ_CASCADE_NARROW=1 AQZ_BAND_MIS_MAX=4 AQZ_BAND_MIS_SEG=0 AQZ_UNITS_PER_WAVE=2 \
    AQZ_LIB_PATH=$PWD/tools/divergent/lib_divdbg.so timeout -k 10 300 python -u tests/narrow_dbg.py > $OUT/dbg_divdbg.log 2>&1
  rc=$?
  echo "== divdbg rc=$rc AQZDBG lines: $(grep -c AQZDBG $OUT/dbg_divdbg.log)"
  grep "differing" $OUT/dbg_divdbg.log
  grep AQZDBG $OUT/dbg_divdbg.log | head -12
  [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in product masked; do
    lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
    [ $v = masked ] && lib=$PWD/tools/divergent/lib_masked.so
    for spec in "4096x4096_f32 5079x3001 mean" "4096x4096_f32 1025x4000 mean" "4096x4096_f32 5079x3001 max" \
                "512x512_u8 1923x1081 mean" "512x512_u8 1923x1081 decimate"; do
      set -- $spec
      f=$OUT/ab_${v}_${1}_${2}_${3}_$rep
      AQZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload $1 --shape $2 --method $3 --steps 20 --warmup 5 \
        --cpu-seconds 0 --e2e-frames 0 --no-pmc > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));r=d['roofline'];print('$v $1 $2 $3 rep $rep', r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])"
    done
  done
done
echo "== done"
