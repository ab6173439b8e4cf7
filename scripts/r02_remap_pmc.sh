#!/bin/bash
# Read requests (TCC_EA0_RDREQ_sum) of 3000^2 / 5472x3648 / 4096^2 cascades
# with and without the XCD-contiguous block order: does cross-XCD sharing of
# the 128-B lines at wave boundaries explain the read excess?
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
for shape in 3000x3000 5472x3648 4096x4096; do for t in "" "--tiled"; do for r in 0 1; do
  name=rq_${shape}${t:+_tiled}_r$r
  rm -rf $OUT/$name
  AQZ_XCD_REMAP=$r timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/$name -o run -- \
    python3 bench.py --pmc-child --steps 2 --warmup 1 --shape $shape $t > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; exit 1; }
  python3 - "$OUT/$name" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = {}
for r in csv.DictReader(open(f)):
    if "cascade_kernel" in r["Kernel_Name"]:
        v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(sys.argv[1].split("/")[-1], {k: int(sum(x) / len(x)) for k, x in v.items()})
PY
done; done; done
echo "== done"
