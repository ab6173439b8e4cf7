#!/bin/bash
# Round-2 GPU session: full GPU suite, then a sweep of the row-major and
# chunk-tiled cascades over aligned and burst-splitting frame shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --steps 30 --warmup 5"
rm -f $OUT/sweep_r02.jsonl
for args in "" "--tiled" "--workload 2048x2048_u16" "--workload 2048x2048_u16 --tiled" \
            "--shape 5472x3648" "--shape 5472x3648 --tiled" "--shape 3000x3000" "--shape 3000x3000 --tiled" \
            "--shape 4100x4100" "--shape 4100x4100 --tiled" "--shape 2000x2000" "--shape 2000x2000 --tiled" \
            "--workload 4096x4096_f32" "--workload 4096x4096_f32 --tiled" "--workload 512x512_u8" "--workload 512x512_u8 --tiled"; do
  timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { echo "FAIL $args"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$args'.ljust(36),d['value'],d['config']['check'][:9],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))"
  cat $OUT/b.json >> $OUT/sweep_r02.jsonl
done
echo "== done"
