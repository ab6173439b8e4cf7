#!/bin/bash
# Round-2 GPU session: per-channel TCC read requests of the volume kernel
# (config V, Decimate vs Mean), and the TCC read-request size mix of
# burst-splitting frames (calibrating FETCH_SIZE's x2 for them).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
run_pmc() { # name counters... -- bench args
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  rm -rf $OUT/pmc_$name
  timeout -s KILL 120 rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d $OUT/pmc_$name -o run -- \
    python3 bench.py --pmc-child --steps 2 --warmup 1 "$@" > $OUT/pmc_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$name.log; return 1; }
  f=$(find $OUT/pmc_$name -name "*counter_collection.csv" | head -1); head -3 "$f" | cut -c1-400; wc -l "$f"
}
run_pmc vol_dec_ch TCC_EA0_RDREQ -- --workload 1024x1024x256_u16 --method decimate || exit 1
run_pmc vol_mean_ch TCC_EA0_RDREQ -- --workload 1024x1024x256_u16 --method mean || exit 1
run_pmc vol2048_dec_ch TCC_EA0_RDREQ -- --workload 1024x1024x256_u16 --method decimate --shape 2048x2048 || exit 1
run_pmc mix3000 TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum -- --shape 3000x3000 --tiled || exit 1
run_pmc mix4096 TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum -- --tiled || exit 1
echo "== done"
