#!/bin/bash
# Headline config under every downsampling method ("also run
# Decimate/Min/Max"); JSON lines into gpurun_out/methods/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/methods
for w in ${WORKLOADS:-4096x4096_u16}; do
  for m in decimate mean min max; do
    timeout -k 10 300 python bench.py --workload "$w" --method "$m" --cpu-seconds "${CPU_S:-3}" \
      --e2e-frames 0 ${BENCH_ARGS:-} > "gpurun_out/methods/${w}_$m.json" 2> "gpurun_out/methods/${w}_$m.err"
    rc=$?; echo "$w $m rc=$rc"
    [ $rc -eq 0 ] || { tail -20 "gpurun_out/methods/${w}_$m.err"; exit $rc; }
  done
done
