#!/bin/bash
# round 4: full GPU suite (reference-made vectors, the executed adapter)
set -euo pipefail
out=gpurun_out/r04_check
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $out/gpu_tests.log 2>&1
