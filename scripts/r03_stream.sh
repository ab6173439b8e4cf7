#!/bin/bash
# Round 3: streaming tiled takes (one-pass tiled cascade vs tile pass) and the
# async-overlap leg; parity first.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03_stream
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread -k "tiled or async" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for mode in 0 1; do
  AQZ_STREAM_TILE_PASS=$mode timeout -k 10 400 python bench.py --steps 10 --warmup 3 \
    --cpu-seconds 0 --no-pmc --e2e-frames 48 > "$OUT/bench_tilepass$mode.json" 2> "$OUT/bench_tilepass$mode.err" \
    || { tail -20 "$OUT/bench_tilepass$mode.err"; exit 1; }
  python - "$OUT/bench_tilepass$mode.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["e2e"]
print({k: e.get(k) for k in ("ms_per_frame", "tiled_take_ms_per_frame", "tiled_one_pass_runs")},
      e.get("async_overlap"))
PY
done
