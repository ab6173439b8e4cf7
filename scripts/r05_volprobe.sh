#!/bin/bash
# Round 5: volume Decimate (config V) access-shape A/B:
# tools/volume_probe.py's variants beside the library's volume_kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_volprobe; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/volume_probe.py --json $OUT/variants.jsonl > $OUT/probe.log 2>&1 || { tail -30 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
