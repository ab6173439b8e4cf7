#!/bin/bash
# Round 4: after taking the tiled cascade out of the units-per-wave loop —
# tiled/row-major GPU tests, then camera shapes and the headline, row-major
# and tiled, with PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_tiledfix; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
sed -i "s#OUT=gpurun_out/r04_shapes#OUT=gpurun_out/r04_tiledfix/shapes#" scripts/r04_shapes.sh
bash scripts/r04_shapes.sh
