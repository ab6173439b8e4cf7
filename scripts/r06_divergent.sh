#!/bin/bash
# Round 6: the round-5 lane-divergent NaN fix-up (tools/divergent/build.sh)
# under compiler switches that isolate the failing pass; the fuzz suite and
# the per-output dump (tests/narrow_dbg.py) for each variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_divergent; mkdir -p $OUT
export TMPDIR=/tmp
for v in div wz; do
  AQZ_LIB_PATH=$PWD/tools/divergent/lib_$v.so timeout -k 10 300 python -u -m pytest -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_fuzz.py -k "device_batch or stream" \
    > $OUT/fuzz_$v.log 2>&1
  rc=$?
  echo "$v: rc=$rc $(tail -1 $OUT/fuzz_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
AQZ_LIB_PATH=$PWD/tools/divergent/lib_div.so timeout -k 10 300 python -u tests/narrow_dbg.py > $OUT/dbg_div.log 2>&1 || exit $?
grep "differing" $OUT/dbg_div.log || true
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_reference_vectors.py tests/test_gpu_adapter.py -k "example" > $OUT/example.log 2>&1
rc=$?; echo "example vectors: rc=$rc $(tail -1 $OUT/example.log)"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_node.py tests/test_gpu_adapter.py -k "node or Node or recycle" > $OUT/node.log 2>&1
rc=$?; echo "node tests: rc=$rc $(tail -1 $OUT/node.log)"
[ $rc -le 1 ] || exit $rc
grep -h "buffers kept" $OUT/node.log | head -3
timeout -k 10 300 tools/write_frame_probe 24 2 > $OUT/probe.json 2> $OUT/probe.err
rc=$?; echo "probe: rc=$rc $(cat $OUT/probe.json)"
[ $rc -eq 0 ] || exit $rc
# then the V Decimate counters (scripts/r06_vdec_pmc.sh), same box
bash scripts/r06_vdec_pmc.sh
