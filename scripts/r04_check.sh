#!/bin/bash
# round 4: full GPU suite (reference-made vectors, the executed adapter, the
# node), then the F-config read-request counters (scripts/r04_f32pmc.sh)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out=gpurun_out/r04_check
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -30 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # test failures: still profile; crashes/timeouts: stop
bash scripts/r04_f32pmc.sh
timeout -k 10 300 python tools/pitch_probe.py --set decimate --json gpurun_out/r04_check/decimate_probe.jsonl \
  > gpurun_out/r04_check/decimate_probe.log 2>&1 || { tail -5 gpurun_out/r04_check/decimate_probe.log; exit 1; }
cat gpurun_out/r04_check/decimate_probe.log
