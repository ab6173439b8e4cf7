#!/bin/bash
# Round 6: V Min/Max with the pass off (product) against on (lib_div: its u16
# shard is the pass-on product build), alternated, plus H Min as control.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_vminmax; mkdir -p $OUT
for rep in 1 2; do
  for v in product passon; do
    lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
    [ $v = passon ] && lib=$PWD/tools/divergent/lib_div.so
    for spec in "1024x1024x256_u16 min" "1024x1024x256_u16 max" "1024x1024x256_u16 decimate" "4096x4096_u16 min"; do
      set -- $spec
      f=$OUT/${v}_${1}_${2}_$rep
      AQZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload $1 --method $2 --steps 20 --warmup 5 --cpu-seconds 0 \
        --e2e-frames 0 --no-pmc > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python -c "import json;d=json.load(open('$f.json'));r=d['roofline'];print('$v $1 $2 rep $rep', r['avg_launch_us'], r['frac'], d['config']['check'][:9])" | tee -a $OUT/summary.txt
    done
  done
done
echo "== done"
