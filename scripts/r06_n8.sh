#!/bin/bash
# Round 6: the N > 1 bench path rehearsed at world size 8 on
# the one-GPU box (gloo, all eight ranks on GPU 0), the driver's own command
# shape; wall time against the driver's 600 s bench limit.  Also N = 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_n8; mkdir -p $OUT
export TMPDIR=/tmp AQZ_DIST_BACKEND=gloo
for n in 2 8; do
  t0=$(date +%s.%N)
  timeout -k 10 700 python bench.py --gpus $n --steps 20 --warmup 5 > $OUT/gpus$n.json 2> $OUT/gpus$n.err
  rc=$?
  t1=$(date +%s.%N)
  echo "gpus $n rc=$rc wall_s=$(python -c "print(round($t1-$t0,1))")" | tee $OUT/gpus$n.wall
  [ $rc -eq 0 ] || { tail -30 $OUT/gpus$n.err; exit $rc; }
  python -c "import json;t=open('$OUT/gpus$n.json').read();assert t.count(chr(10)) == 1 and t.startswith('{'), 'stdout is not one JSON line';d=json.loads(t);e=d['e2e'];print(d['n_gpus'], d['value'], d['ms_per_step'], d.get('rehearsal'), d['config']['parallelism'], json.dumps(e.get('node_device_batch'))[:400])"
done
echo "== done"
