#!/bin/bash
# Round 6: the headline kernel's HBM traffic from rocprofv3 --pmc directly
# (one counter per pass, as the guide prescribes), beside the bench line's
# own child passes: FETCH_SIZE (KiB, x2 on gfx950) and WRITE_SIZE (KiB) per
# launch of the dominant kernel, against the algorithmic bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_pmc; mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o pmc -- \
    python3 bench.py --pmc-child --steps 5 --warmup 2 > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
done
python3 - $OUT <<'PY' | tee $OUT/pmc_summary.txt
import csv, glob, sys, collections
out = sys.argv[1]
alg = 2860515328  # algorithmic bytes per headline launch
tot = {}
for c, scale in (("FETCH_SIZE", 2048), ("WRITE_SIZE", 1024)):
    f = glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "cascade_band_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
            per[r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
    v = sorted(per.values())
    mid = v[len(v) // 2] * scale
    tot[c] = mid
    print(f"{c}: {len(v)} launches, median {mid / 1e9:.4f} GB per launch (x{scale} B)")
print(f"traffic per launch {sum(tot.values()) / 1e9:.4f} GB; algorithmic {alg / 1e9:.4f} GB; "
      f"ratio {sum(tot.values()) / alg:.5f}")
PY
echo "== done"
