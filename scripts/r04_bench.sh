#!/bin/bash
# Round 4: the default bench line (headline + roofline + PMC traffic + the
# reference-itself cpu_baseline + e2e incl. the node leg), its rocprofv3
# kernel-trace summary, and the smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04_bench; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
start=$(date +%s)
timeout -k 10 600 python bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || { tail -20 $OUT/bench_headline.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04_bench/bench_headline.json"))
r = d["roofline"]; c = d["cpu_baseline"]; e = d["e2e"]
print(d["value"], d["ms_per_step"], r["frac"], r["traffic"], r.get("same_mix_ceiling", {}).get("frac_of_ceiling"))
print("cpu", c["kind"], c["value"], c["ms_per_frame"], c.get("port"), c.get("reference_over_port_time"), c.get("parallel"))
print("e2e", e.get("ms_per_frame"), e.get("pipelined", {}).get("value"), e.get("node"))
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-check --no-pmc > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats*" | head -3
echo "== done"
