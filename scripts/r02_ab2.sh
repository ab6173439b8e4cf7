#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check --steps 30 --warmup 5"
run() { # label env... -- args
  local label=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py $B "$@" > $OUT/b.json 2> $OUT/b.err || { echo "FAIL $label"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$label'.ljust(40),d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))" | tee -a $OUT/ab2.log
}
for rep in 1 2; do
run "headline" X=1 -- 
run "headline tiled" X=1 -- --tiled
run "512 u8 tiled flagnt0" AQZ_FLAG_NT=0 -- --workload 512x512_u8 --tiled
run "512 u8 tiled flagnt1" AQZ_FLAG_NT=1 -- --workload 512x512_u8 --tiled
run "headline tiled flagnt1" AQZ_FLAG_NT=1 -- --tiled
run "2000 rowmajor(band) nt-auto" X=1 -- --shape 2000x2000
run "2000 rowmajor(band) nt1" AQZ_LOAD_NT=1 -- --shape 2000x2000
run "3000 rowmajor" X=1 -- --shape 3000x3000
run "3000 tiled" X=1 -- --shape 3000x3000 --tiled
done
