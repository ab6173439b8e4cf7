#!/bin/bash
# Round 4: the chunk-tiled batch ran slower than in round 3 (3000^2 539 ->
# 710 us): per-launch vs span events, and the kernel trace of one tiled run.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_tiledreg; mkdir -p $OUT
export TMPDIR=/tmp
for sh in 3000x3000 4096x4096; do
  for pl in "" "--per-launch-events"; do
    timeout -k 10 300 python bench.py --shape $sh --tiled $pl --steps 20 --warmup 5 --cpu-seconds 0 --e2e-frames 0 --no-pmc \
      > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('$sh', '$pl', d['ms_per_step'], r['avg_launch_us'], r['frac'])" | tee -a $OUT/ab.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --shape 3000x3000 --tiled --steps 10 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04_tiledreg/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-12:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(r["Kernel_Name"][:90], round((e - s) / 1e3, 1), "gap", None if prev is None else round((s - prev) / 1e3, 1), r["Grid_Size_X"], r["Workgroup_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"])
    prev = e
PY
echo "== done"
