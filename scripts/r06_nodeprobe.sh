#!/bin/bash
# Round 6: synchronous drop-in vs node mode over the same
# frame sets (tools/node_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_nodeprobe; mkdir -p $OUT
timeout -k 10 400 python -u tools/node_probe.py > $OUT/node_probe.json 2> $OUT/node_probe.err || { tail -20 $OUT/node_probe.err; exit 1; }
cat $OUT/node_probe.json
echo "== done"
