#!/bin/bash
# Round 5: the default line's e2e.node_device_batch leg (config F's shape of
# work through aqz_node_run_device_batch over the ranks' / visible GPUs) at
# N=1 and, rehearsed with gloo on the one-GPU box, N=2.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_ndb; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/gpus1.json 2> $OUT/gpus1.err || { tail -30 $OUT/gpus1.err; exit 1; }
python -c "import json;t=open('$OUT/gpus1.json').read();assert t.count(chr(10)) == 1 and t.startswith('{');d=json.loads(t);print(d['value'], d['roofline']['frac'], json.dumps(d['e2e']['node_device_batch']))"
AQZ_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --e2e-frames 8 > $OUT/gpus2.json 2> $OUT/gpus2.err || { tail -30 $OUT/gpus2.err; exit 1; }
python -c "import json;t=open('$OUT/gpus2.json').read();assert t.count(chr(10)) == 1 and t.startswith('{'), 'stdout is not one JSON line';d=json.loads(t);print(d['n_gpus'], d['value'], d.get('rehearsal'), json.dumps(d['e2e']['node_device_batch']))"
echo "== done"
