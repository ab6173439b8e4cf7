#!/bin/bash
# Tiled takes: parity (streaming takes, tiled batches incl. the chain
# sequence), then the host-to-host breakdown of the drop-in calls.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/takes; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiled.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/e2e_takes.py > $OUT/e2e_takes.log 2>&1 || { tail -20 $OUT/e2e_takes.log; exit 1; }
grep -v amdgpu.ids $OUT/e2e_takes.log
echo "== done"
