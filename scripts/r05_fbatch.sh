#!/bin/bash
# Round 5: launch size A/B (default config F, 4096^2 f32; $W, $BATCHES and
# $METHODS override): 16/32/64/128 frames per launch, two passes, with the same-mix ceiling each line measures.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_fbatch; mkdir -p $OUT
export TMPDIR=/tmp
W=${W:-4096x4096_f32}
for pass in 1 2; do
  for b in ${BATCHES:-16 32 64 128}; do
    for m in ${METHODS:-mean max}; do
      timeout -k 10 300 python bench.py --workload $W --method $m --batch $b --steps 20 --warmup 5 \
        --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/${W}_${m}_b${b}_p$pass.json 2> $OUT/${W}_${m}_b${b}_p$pass.err || { tail -20 $OUT/${W}_${m}_b${b}_p$pass.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/${W}_${m}_b${b}_p$pass.json'));r=d['roofline'];print('$W', 'pass $pass', '$m', 'batch $b', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('GBps'), r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), d['config']['check'])" | tee -a $OUT/ab.log
    done
  done
done
echo "== done"
