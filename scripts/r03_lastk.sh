#!/bin/bash
# Round 3: band stores by the last K waves to arrive ($AQZ_BAND_LAST=K; 0 is
# the barrier form).  Parity for K = 2 with every level of misaligned 5-8-tile
# bands staged, then A/B over K on misaligned and aligned band shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_lastk; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_BAND_LAST=2 AQZ_BAND_FORCE=15 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch" --timeout 120 --timeout-method thread > $OUT/pytest_k2_force.log 2>&1 || { tail -30 $OUT/pytest_k2_force.log; exit 1; }
tail -1 $OUT/pytest_k2_force.log
AQZ_BAND_LAST=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "device_batch or headline" --timeout 120 --timeout-method thread > $OUT/pytest_k3.log 2>&1 || { tail -30 $OUT/pytest_k3.log; exit 1; }
tail -1 $OUT/pytest_k3.log
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for k in 0 2 4; do
    b headline "AQZ_BAND_LAST=$k"
    b f32_mean "AQZ_BAND_LAST=$k" --workload 4096x4096_f32
  done
  for k in 0 1 2 3; do
    b 2000 "AQZ_BAND_LAST=$k" --shape 2000x2000
  done
  for sh in 3000x3000 2600x2600 4000x3000; do
    b $sh "X=0" --shape $sh
    for k in 1 2 3; do
      b $sh "AQZ_BAND_FORCE=15 AQZ_BAND_LAST=$k" --shape $sh
    done
  done
done
echo "== done"
