#!/bin/bash
# Round 6: what would building the product with the
# VGPR live-range optimisation off cost?  lib_prodnolr (every object built
# with -mllvm -amdgpu-opt-vgpr-liverange=false) against the product:
# parity (the fuzz suite) and kernel time on H, F, C2, C1b and V, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_prodnolr; mkdir -p $OUT
AQZ_LIB_PATH=$PWD/tools/divergent/lib_prodnolr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/fuzz.log 2>&1; echo "fuzz rc=$? $(tail -1 $OUT/fuzz.log)"
for rep in 1 2; do
  for v in product prodnolr; do
    lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
    [ $v = prodnolr ] && lib=$PWD/tools/divergent/lib_prodnolr.so
    for spec in "4096x4096_u16 mean" "4096x4096_f32 mean" "2048x2048_u16 mean" "512x512_u8 decimate" "1024x1024x256_u16 mean"; do
      set -- $spec
      f=$OUT/${v}_${1}_${2}_$rep
      AQZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload $1 --method $2 --steps 20 --warmup 5 --cpu-seconds 0 \
        --e2e-frames 0 --no-pmc > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));r=d['roofline'];print('$v $1 $2 rep $rep', r['avg_launch_us'], r['frac'], d['config']['check'][:9])" | tee -a $OUT/summary.txt
    done
  done
done
echo "== done"
