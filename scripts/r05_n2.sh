#!/bin/bash
# Round 5: the N > 1 bench paths rehearsed on the one-GPU box with gloo
# (both ranks on GPU 0): the default frame-sharded line, and --xgmi-scatter
# with the node's handles on 0,0 (rank 0 drives, rank 1 waits).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_n2; mkdir -p $OUT
export TMPDIR=/tmp AQZ_DIST_BACKEND=gloo
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --e2e-frames 8 > $OUT/gpus2.json 2> $OUT/gpus2.err || { tail -30 $OUT/gpus2.err; exit 1; }
python -c "import json;t=open('$OUT/gpus2.json').read();assert t.count(chr(10)) == 1 and t.startswith('{'), 'stdout is not one JSON line';d=json.loads(t);print(d['n_gpus'], d['value'], d.get('rehearsal'), d['config']['parallelism'], d['library'], json.dumps(d['e2e']['node'])[:300])"
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --e2e-frames 0 --workload 4096x4096_f32 \
  --xgmi-scatter --node-devices 0,0 > $OUT/xgmi2.json 2> $OUT/xgmi2.err || { tail -30 $OUT/xgmi2.err; exit 1; }
python -c "import json;t=open('$OUT/xgmi2.json').read();assert t.count(chr(10)) == 1 and t.startswith('{'), 'stdout is not one JSON line';d=json.loads(t);print(d['n_gpus'], d['value'], d['ms_per_step'], d.get('rehearsal'), d['config']['check'], d['config']['parallelism'], json.dumps(d['xgmi_node'])[:300])"
echo "== done"
