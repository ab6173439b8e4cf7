#!/bin/bash
# Round 3: band-aligned workgroups with the XCD-contiguous block order (so
# neighbouring bands share an L2) — A/B and partial-write counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_remap; mkdir -p $OUT
export TMPDIR=/tmp
b() { # label env args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc "$@" > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$lab', '$e', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/ab.log
}
for i in 1 2; do
  for sh in 3000x3000 2600x2600 5472x3648 2112x2048; do
    b "$sh" "X=0" --shape $sh
    b "$sh" "AQZ_XCD_REMAP=1" --shape $sh
    b "$sh" "AQZ_XCD_REMAP=1 AQZ_STORE_WB=15" --shape $sh
  done
done
for e in "X=0" "AQZ_XCD_REMAP=1"; do
  env $e timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_$e -o pmc -- \
    python3 bench.py --pmc-child --steps 3 --warmup 1 --shape 3000x3000 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
  python3 - "$OUT/pmc_$e" "$e" <<'PY' | tee -a $OUT/pmc_summary.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "cascade" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("3000x3000", sys.argv[2], {k: round(sum(v[1:]) / max(1, len(v) - 1)) for k, v in acc.items()})
PY
done
echo "== done"
