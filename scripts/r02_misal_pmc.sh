#!/bin/bash
# Counters for misaligned staging (3000^2 u16, level 1 staged) against the
# aligned staged headline and the direct 3000^2 launch: LDS bank conflicts,
# wave stall buckets, L2->EA write requests.  One counter set per pass.  r02u/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r02u; mkdir -p $OUT
export TMPDIR=/tmp
run() { # tag env counters bench-args
  local tag=$1 e=$2 c=$3; shift 3
  env $e timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$tag -o pmc -- \
    python3 bench.py --pmc-child --steps 3 --warmup 1 "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$OUT/$tag" "$tag" <<'PY'
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
C3="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
for args in "--shape 3000x3000" ; do
  for e in "X=0" "AQZ_BAND_FORCE=1"; do
    for c in "$C1" "$C2" "$C3"; do
      tag="m$(echo $e | tr -dc 'A-Z0-9')_$(echo $c | cut -c1-12 | tr -dc 'A-Z_')"
      run "$tag" "$e" "$c" $args
    done
  done
done
for c in "$C1" "$C2" "$C3"; do
  run "h_$(echo $c | cut -c1-12 | tr -dc 'A-Z_')" "X=0" "$c"
done
echo "== done"
