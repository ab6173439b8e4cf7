#!/bin/bash
# Round 5: the fuzz cases that fail with 16-byte f32 tiles, under switches
# that isolate the store path (AQZ_BAND_WG=0: no band workgroups;
# AQZ_CASCADE_NARROW=0: wide tiles; AQZ_UNITS_PER_WAVE=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_narrow_dbg; mkdir -p $OUT
export TMPDIR=/tmp
K="test_fuzz_device_batch and (4 or 86 or 174 or 192)"
for cfg in "AQZ_UNUSED=0" "AQZ_CASCADE_NARROW=0" "AQZ_BAND_WG=0" "AQZ_UNITS_PER_WAVE=1" "AQZ_LOAD_NT=1" "AQZ_LOAD_NT=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_fuzz.py -k "$K" > $OUT/$cfg.log 2>&1
  echo "$cfg: $(tail -1 $OUT/$cfg.log)"
done
python - <<'PY'
import sys; sys.path.insert(0, "tests")
import test_gpu_fuzz as t
for c in (4, 86, 174, 192):
    try:
        print(c, t._case(c) if hasattr(t, "_case") else "")
    except Exception as e:
        print(c, "?", e)
PY
echo "== done"
