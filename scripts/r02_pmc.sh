#!/bin/bash
# Round-2 GPU session: full GPU suite, PMC traffic of the tiled and row-major
# cascades on aligned and burst-splitting frame shapes, and the counter list
# (per-channel TCC counters for the volume Decimate question).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
echo "== full gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
export TMPDIR=/tmp
echo "== counters"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/rocprof_list_avail.txt 2>&1 || true
grep -n "TCC_EA0_RDREQ\b\|TCC_EA0_RDREQ\[" $OUT/rocprof_list_avail.txt | head -5
B="--cpu-seconds 0 --e2e-frames 0 --steps 20 --warmup 3"
for args in "--tiled" "--shape 3000x3000 --tiled" "--shape 3000x3000" "--shape 5472x3648 --tiled" "--shape 5472x3648"; do
  echo "== bench+pmc $args"
  timeout -k 10 400 python bench.py $B $args > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];t=r.get('traffic_detail') or {};print(d['value'],r['avg_launch_us'],r['frac'],r.get('same_mix_ceiling',{}).get('frac_of_ceiling'),'alg',r['alg_bytes_per_launch'],'pmc',r['traffic'],'rd',t.get('read_bytes'),'wr',t.get('write_bytes'))"
  cat $OUT/b.json >> $OUT/bench_pmc_r02.jsonl
done
echo "== done"
