#!/bin/bash
# Round 6: the whole GPU suite twice more on the final tree (flakiness check
# after the one-off wrong pixel of a probe build).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_suite_rep; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu_$rep.log 2>&1 || { tail -40 $OUT/pytest_gpu_$rep.log; exit 1; }
  tail -1 $OUT/pytest_gpu_$rep.log
done
echo "== done"
