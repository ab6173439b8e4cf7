#!/bin/bash
# Round 5: volume Decimate launch size (256/512/1024 planes = 1/2/4 volumes)
# against the load policy and units per wave ($AQZ_VOLUME_NT, $AQZ_VOLUME_UPW).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_vdec; mkdir -p $OUT
export TMPDIR=/tmp
for pass in 1 2; do
  for b in 256 512 1024; do
    for v in "0 2" "1 2" "0 1" "1 1"; do
      set -- $v
      AQZ_VOLUME_NT=$1 AQZ_VOLUME_UPW=$2 timeout -k 10 300 python bench.py --workload 1024x1024x256_u16 --method decimate --batch $b \
        --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/d_b${b}_nt$1_upw$2_p$pass.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
      python -c "import json;d=json.load(open('$OUT/d_b${b}_nt$1_upw$2_p$pass.json'));r=d['roofline'];print('pass $pass', 'planes $b', 'nt $1', 'upw $2', r['avg_launch_us'], r['frac'], d['config']['check'])" | tee -a $OUT/ab.log
    done
  done
done
echo "== done"
