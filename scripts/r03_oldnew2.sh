#!/bin/bash
# Round 3: rowwise segments as their own band-kernel instantiation (whole
# bands keep their code) against the tree before the segments (cad98a9, in
# _ab_old/), same box, alternating, two rounds; full GPU suite first.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out/r03_oldnew2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() { # label dir args...
  local lab=$1 d=$2; shift 2
  (cd $d && timeout -k 10 180 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err) || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$(basename $d)', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for d in $ROOTDIR $ROOTDIR/_ab_old; do
    b u16_3000x3000 $d --shape 3000x3000
    b u16_2600x2600 $d --shape 2600x2600
    b u16_2000x2000 $d --shape 2000x2000
    b u16_6000x4000 $d --shape 6000x4000
    b f32_5472x3648 $d --workload 4096x4096_f32 --shape 5472x3648
    b headline $d
  done
done
echo "== done"
