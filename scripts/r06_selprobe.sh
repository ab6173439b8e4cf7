#!/bin/bash
# Round 6: the select form's wrong u16 pixel (fuzz case
# 181).  For each shard-1 (u16) probe build and the product: case 181 200
# times in one process, then 10 fresh processes that each run cases 170-180
# once and 181 once (tests/fuzz_repeat.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${R06_OUT:-r06_selprobe}; mkdir -p $OUT
for v in ${VARIANTS:-u16rowsel u16rowselwz u16srcsel u16rowsel32 product}; do
  lib=$PWD/tools/divergent/lib_$v.so
  [ $v = product ] && lib=$PWD/acquire-zarr_amd/libaqz_downsampler.so
  [ -f $lib ] || { echo "$v: not built"; continue; }
  AQZ_LIB_PATH=$lib timeout -k 10 200 python -u tests/fuzz_repeat.py --cases 181 --reps ${REPS:-200} > $OUT/${v}_inproc.json 2> $OUT/${v}_inproc.err \
    || { tail -5 $OUT/${v}_inproc.err; exit 1; }
  echo "$v in-process: $(cat $OUT/${v}_inproc.json)"
  fresh=0
  for i in $(seq 1 10); do
    AQZ_LIB_PATH=$lib timeout -k 10 200 python -u tests/fuzz_repeat.py --cases 181 --reps 1 --from 170 > $OUT/${v}_fresh_$i.json 2>> $OUT/${v}_fresh.err \
      || { tail -5 $OUT/${v}_fresh.err; exit 1; }
    python -c "import json,sys;d=json.load(open('$OUT/${v}_fresh_$i.json'));sys.exit(0 if d['181'][0] else 1)" && fresh=$((fresh+1))
  done
  echo "$v fresh processes with a wrong pixel: $fresh of 10" | tee -a $OUT/summary.txt
done
echo "== done"
