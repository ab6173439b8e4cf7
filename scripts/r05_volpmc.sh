#!/bin/bash
# Round 5, VERDICT r4 item 2 (counter evidence): the fused 2x2x2 volume
# Decimate launch with nontemporal vs plain loads ($AQZ_VOLUME_NT=1/0) and
# one vs two units per wave ($AQZ_VOLUME_UPW).  Per volume_kernel launch:
# TCC read requests by size, TCC hit/miss, and the DRAM-side 32-B reads;
# Mean as the dense-read calibration.  Each pass is a run of its own.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${R05_OUT:-r05_volpmc}; mkdir -p $OUT
export TMPDIR=/tmp
run() { # tag counters bench-args
  local tag=$1 c=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$tag -o pmc -- \
    python3 bench.py --pmc-child --steps 3 --warmup 1 --no-check "$@" > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  python3 - "$OUT/$tag" "$tag" <<'PY' | tee -a $OUT/pmc_summary.txt
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "volume_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(v[1:]) / max(1, len(v) - 1)) for k, v in sorted(acc.items())})
PY
}
CA="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
CB="TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum"
CC="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
W="--workload 1024x1024x256_u16"
for cfg in "1 1" "0 1" "1 2" "0 2"; do
  set -- $cfg
  tag="dec_nt$1_upw$2"
  AQZ_VOLUME_NT=$1 AQZ_VOLUME_UPW=$2 run ${tag}_A "$CA" $W --method decimate
  AQZ_VOLUME_NT=$1 AQZ_VOLUME_UPW=$2 run ${tag}_B "$CB" $W --method decimate
  AQZ_VOLUME_NT=$1 AQZ_VOLUME_UPW=$2 run ${tag}_C "$CC" $W --method decimate
done
run mean_default_A "$CA" $W --method mean
run mean_default_B "$CB" $W --method mean
for cfg in "1 1" "0 1" "1 2" "0 2"; do
  set -- $cfg
  AQZ_VOLUME_NT=$1 AQZ_VOLUME_UPW=$2 timeout -k 10 300 python bench.py $W --method decimate --steps 20 --warmup 5 \
    --cpu-seconds 0 --e2e-frames 0 > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];print('nt=$1 upw=$2', r['avg_launch_us'], r['frac'], r['same_mix_ceiling']['frac_of_ceiling'], r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/ab.log
done
echo "== done"
