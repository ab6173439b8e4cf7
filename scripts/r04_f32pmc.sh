#!/bin/bash
# Round 4, VERDICT r3 item 2: where do F-config (4096^2 f32) Min/Max fetch
# 2-3% more than the algorithmic bytes?  Per-kernel TCC read-request counters
# by request size, and the DRAM-side 32-B read count (exact bytes), for every
# method on F and for the u16 headline (calibration: 16 B/lane streaming).
# $AQZ_LOAD_NT=0/1 A/B of the load cache policy.  One rocprofv3 pass per
# counter set (<= 4 TCC counters each).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_f32pmc; mkdir -p $OUT
export TMPDIR=/tmp
run() { # tag counters bench-args
  local tag=$1 c=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$tag -o pmc -- \
    python3 bench.py --pmc-child --steps 3 --warmup 1 "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$OUT/$tag" "$tag" <<'PY' | tee -a $OUT/pmc_summary.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
names = set()
for r in csv.DictReader(open(f)):
    if "cascade" in r["Kernel_Name"] or "volume" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        names.add(r["Kernel_Name"].split("(")[0][:90])
print(sys.argv[2], {k: round(sum(v[1:]) / max(1, len(v) - 1)) for k, v in acc.items()}, sorted(names)[:2])
PY
}
CA="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
CB="TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum"
for nt in "" 0; do
  for m in mean max min decimate; do
    AQZ_LOAD_NT=$nt run "f32_${m}_nt${nt:-def}_A" "$CA" --workload 4096x4096_f32 --method $m
    AQZ_LOAD_NT=$nt run "f32_${m}_nt${nt:-def}_B" "$CB" --workload 4096x4096_f32 --method $m
  done
done
run "u16_mean_A" "$CA" --workload 4096x4096_u16 --method mean
run "u16_mean_B" "$CB" --workload 4096x4096_u16 --method mean
for nt in "" 0; do
  for m in max mean; do
    AQZ_LOAD_NT=$nt timeout -k 10 120 python bench.py --workload 4096x4096_f32 --method $m --steps 20 --warmup 5 \
      --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('nt=${nt:-def}', '$m', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], d['config']['check'])" | tee -a $OUT/ab.log
  done
done
echo "== done"
