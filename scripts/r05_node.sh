#!/bin/bash
# Round 5: the node's device-resident batch (aqz_node_run_device_batch,
# VERDICT r4 item 3) against the reference digests and the oracle, in place
# and through the staged (remote-GPU) path; the existing node tests; the
# drop-in's node mode and async-then-sync mode (ADVICE
# r4); then bench.py --xgmi-scatter rehearsed on one GPU (handles 0,0, every
# block staged) and the default line with the C2 filesystem-sink leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_node; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_node_device.py tests/test_gpu_node.py tests/test_gpu_adapter.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload 4096x4096_f32 --xgmi-scatter --node-devices 0,0 --stage-all \
  --steps 10 --warmup 3 --cpu-seconds 0 --e2e-frames 0 --no-pmc > $OUT/xgmi_rehearsal.json 2> $OUT/xgmi_rehearsal.err || { tail -30 $OUT/xgmi_rehearsal.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/xgmi_rehearsal.json'));print(d['value'], d['ms_per_step'], d['config']['check'], d['roofline']['frac'], json.dumps(d['xgmi_node']))"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['roofline']['frac'], json.dumps(d['e2e']['c2_filesystem_sink']))"
echo "== done"
