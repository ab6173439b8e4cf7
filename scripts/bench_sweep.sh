#!/bin/bash
# Bench every BASELINE config on one GPU; JSON lines into gpurun_out/sweep/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/sweep
for w in ${WORKLOADS:-4096x4096_u16 4096x4096_f32 2048x2048_u16 512x512_u8 1024x1024x256_u16}; do
  timeout -k 10 300 python bench.py --workload "$w" --cpu-seconds "${CPU_S:-5}" ${BENCH_ARGS:-} \
    > "gpurun_out/sweep/$w.json" 2> "gpurun_out/sweep/$w.err"
  rc=$?; echo "$w rc=$rc"; cat "gpurun_out/sweep/$w.json"
  [ $rc -eq 0 ] || { tail -20 "gpurun_out/sweep/$w.err"; exit $rc; }
done
