#!/bin/bash
# One GPU-box session: smoke, C++ + pytest GPU parity, bench, rocprof stats.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
STEPS="${STEPS:-smoke cpp pytest bench prof}"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

for s in $STEPS; do
  case "$s" in
  smoke)
    echo "== smoke"
    timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -5 "$OUT/smoke.log"
    [ $rc -eq 0 ] || exit $rc ;;
  cpp)
    echo "== cpp"
    for t in test_downsampler test_downsampler_odd_z; do
      timeout -k 10 120 tests/cpp/bin/$t > "$OUT/$t.log" 2>&1
      rc=$?; echo "$t rc=$rc"; tail -3 "$OUT/$t.log"
      if fatal $rc; then exit $rc; fi
    done ;;
  pytest)
    echo "== pytest -m gpu"
    timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=25 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
    if fatal $rc; then exit $rc; fi ;;
  bench)
    echo "== bench"
    timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
    rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
    [ $rc -eq 0 ] || exit $rc ;;
  prof)
    echo "== rocprofv3 kernel-trace"
    export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 \
      --cpu-seconds 0 --e2e-frames 0 --no-check ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
    rc=$?; echo "prof rc=$rc"; tail -3 "$OUT/prof.log"
    find "$OUT/prof" -name "*stats*" | head
    [ $rc -eq 0 ] || exit $rc ;;
  prof2)
    echo "== rocprofv3 kernel-trace, 8(f) kernels"
    export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof2" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 \
      --cpu-seconds 0 --e2e-frames 8 --no-pmc --no-check > "$OUT/prof2.log" 2>&1
    rc=$?; echo "prof2 rc=$rc"; tail -3 "$OUT/prof2.log"
    find "$OUT/prof2" -name "*stats*" | head
    [ $rc -eq 0 ] || exit $rc ;;
  probe)
    echo "== write_frame probe"
    timeout -k 10 300 tools/write_frame_probe ${PROBE_ARGS:-} > "$OUT/write_frame_probe.json" 2> "$OUT/write_frame_probe.err"
    rc=$?; echo "probe rc=$rc"; cat "$OUT/write_frame_probe.json"; tail -3 "$OUT/write_frame_probe.err"
    [ $rc -eq 0 ] || exit $rc ;;
  pmc)
    echo "== rocprofv3 pmc"
    export TMPDIR=/tmp
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run \
        -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 \
        --e2e-frames 0 --no-check ${BENCH_ARGS:-} > "$OUT/pmc_$c.log" 2>&1
      rc=$?; echo "pmc $c rc=$rc"; tail -3 "$OUT/pmc_$c.log"
      [ $rc -eq 0 ] || exit $rc
    done ;;
  esac
done
echo "== done"
