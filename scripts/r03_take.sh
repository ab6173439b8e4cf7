#!/bin/bash
# Round 3: background takes (aqz_ds_add_frame_async_take): parity, then the
# streaming e2e legs of the bench line; then the F config method repeat.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r03_take; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "async or tiled" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-pmc --e2e-frames 48 \
  > $OUT/bench_stream.json 2> $OUT/bench_stream.err || { tail -5 $OUT/bench_stream.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_stream.json'));e=d['e2e'];print({k:e.get(k) for k in ('ms_per_frame','tiled_take_ms_per_frame','async_overlap_ms_per_frame','async_take_ms_per_frame')}, e['async_overlap'])"
bash scripts/r03_f32b.sh
