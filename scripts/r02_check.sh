#!/bin/bash
# Round-2 GPU session: new parity tests, full GPU suite, 2-rank launcher
# rehearsal (gloo, both ranks on GPU 0), config C2 with the filesystem sink.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
echo "== new tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "temporaries or interleave or async" > $OUT/pytest_new.log 2>&1 || { tail -30 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "== bench --gpus 2 (gloo, shared GPU)"
AQZ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --cpu-seconds 0 \
  --e2e-frames 8 --no-pmc > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err || { tail -30 $OUT/bench_gpus2.err; exit 1; }
cat $OUT/bench_gpus2.json
echo "== C2 filesystem sink"
timeout -k 10 400 python bench.py --workload 2048x2048_u16 --sink /tmp/aqz_sink_c2 --e2e-frames 256 \
  --cpu-seconds 5 --no-pmc > $OUT/bench_c2_sink.json 2> $OUT/bench_c2_sink.err || { tail -30 $OUT/bench_c2_sink.err; exit 1; }
cat $OUT/bench_c2_sink.json
echo "== done"
