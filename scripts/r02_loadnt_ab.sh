#!/bin/bash
# A/B: cascade loads with / without the non-temporal hint ($AQZ_LOAD_NT) on
# burst-splitting and aligned frames; read requests counted for each.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
B="--cpu-seconds 0 --e2e-frames 0 --no-pmc --no-check --steps 30 --warmup 5"
for rep in 1 2; do
for args in "--shape 3000x3000 --tiled" "--shape 3000x3000" "--shape 5472x3648 --tiled" "" "--tiled"; do
  for nt in 1 0; do
    AQZ_LOAD_NT=$nt timeout -k 10 200 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('nt=$nt','$args',d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'))" | tee -a $OUT/loadnt_ab.log
  done
done
done
for nt in 1 0; do
  name=rqnt_3000_$nt; rm -rf $OUT/$name
  AQZ_LOAD_NT=$nt timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/$name -o run -- \
    python3 bench.py --pmc-child --steps 2 --warmup 1 --shape 3000x3000 --tiled > $OUT/$name.log 2>&1 || { echo "$name failed"; exit 1; }
  python3 - "$OUT/$name" <<'PY' | tee -a $OUT/loadnt_ab.log
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = {}
for r in csv.DictReader(open(f)):
    if "cascade_kernel" in r["Kernel_Name"]:
        v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(sys.argv[1].split("/")[-1], {k: int(sum(x) / len(x)) for k, x in v.items()})
PY
done
echo "== done"
