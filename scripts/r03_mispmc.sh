#!/bin/bash
# Round 3: counters for misaligned row-major output (band-aligned workgroups)
# against the tiled kernel on the same frames and the aligned headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_mispmc; mkdir -p $OUT
export TMPDIR=/tmp
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
C1="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
C2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
C3="FETCH_SIZE"
C4="WRITE_SIZE"
C5="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES"
for c in "$C1" "$C2" "$C3" "$C4" "$C5"; do
  t=$(echo $c | cut -c1-14 | tr -dc 'A-Z_0-9')
  run "rm3000_$t" "$c" --shape 3000x3000
  run "tl3000_$t" "$c" --shape 3000x3000 --tiled
  run "rm5472_$t" "$c" --shape 5472x3648
  run "head_$t" "$c"
done
echo "== done"
