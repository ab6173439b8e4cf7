#!/bin/bash
# Round 4, VERDICT r3 item 2: F-config (4096^2 f32) Min/Max fetch 2-3% more
# than the algorithmic bytes.  (1) parity of the whole-line (SPLIT) loads:
# the batch/full-size GPU parity tests with $AQZ_SPLIT_LOADS=1;  (2) per-
# kernel TCC read requests by size and the DRAM-side 32-B read count (exact
# bytes) for every method, 32-B-per-lane loads vs SPLIT, and the u16
# headline as calibration;  (3) alternating timing A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_f32pmc; mkdir -p $OUT
export TMPDIR=/tmp
AQZ_SPLIT_LOADS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py \
  tests/test_gpu_fuzz.py -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "batch or full_size or headline or digest or fuzz" > $OUT/split_parity.log 2>&1 || { tail -30 $OUT/split_parity.log; exit 1; }
tail -2 $OUT/split_parity.log
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
        names.add(r["Kernel_Name"].split("(")[0][:60])
print(sys.argv[2], {k: round(sum(v[1:]) / max(1, len(v) - 1)) for k, v in acc.items()}, sorted(names)[:2])
PY
}
CA="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
CB="TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum"
for sp in 0 1; do
  for m in max min mean decimate; do
    AQZ_SPLIT_LOADS=$sp run "f32_${m}_split${sp}_A" "$CA" --workload 4096x4096_f32 --method $m
    AQZ_SPLIT_LOADS=$sp run "f32_${m}_split${sp}_B" "$CB" --workload 4096x4096_f32 --method $m
  done
done
run "u16_mean_A" "$CA" --workload 4096x4096_u16 --method mean
run "u16_mean_B" "$CB" --workload 4096x4096_u16 --method mean
for i in 1 2; do
  for sp in 0 1; do
    for m in max min mean decimate; do
      AQZ_SPLIT_LOADS=$sp timeout -k 10 300 python bench.py --workload 4096x4096_f32 --method $m --steps 20 --warmup 5 \
        --cpu-seconds 0 --e2e-frames 0 > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('split=$sp', '$m', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/ab.log
    done
  done
done
echo "== done"
