#!/bin/bash
# Round 3: F config methods after the vectorised LDS staging writes — three
# alternating rounds against the same-mix ceiling, then counters per method.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_f32b; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for m in max min decimate mean; do
    timeout -k 10 120 python bench.py --workload 4096x4096_f32 --method $m --steps 20 --warmup 5 \
      --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$m', r['avg_launch_us'], r['min_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['same_mix_ceiling']['GBps'], d['config']['check'])" | tee -a $OUT/f32_methods.log
  done
done
run() { # tag counters bench-args
  local tag=$1 c=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$tag -o pmc -- \
    python3 bench.py --pmc-child --steps 3 --warmup 1 "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$OUT/$tag" "$tag" <<'PY' | tee -a $OUT/pmc_summary.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "cascade" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(v[1:]) / max(1, len(v) - 1)) for k, v in acc.items()})
PY
}
C1="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
C2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES"
C3="FETCH_SIZE"
C4="WRITE_SIZE"
for m in max mean; do
  for c in "$C1" "$C2" "$C3" "$C4"; do
    run "${m}_$(echo $c | cut -c1-12 | tr -dc 'A-Z_')" "$c" --workload 4096x4096_f32 --method $m
  done
done
echo "== done"
