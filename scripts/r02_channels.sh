#!/bin/bash
# Round-2 GPU session: per-channel TCC read requests (tools/pmc/tcc_channels.yaml)
# of the volume kernel, Decimate vs Mean, at plane widths 1024 (config V) and
# 512/2048 (tools/volume_shape_probe.py widths).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
Y=$PWD/tools/pmc/tcc_channels.yaml
run() { # name "counters" bench args...
  local name=$1 ctrs=$2; shift 2
  rm -rf $OUT/ch_$name
  timeout -s KILL 90 rocprofv3 -E $Y --pmc $ctrs --output-format csv -d $OUT/ch_$name -o run -- \
    python3 bench.py --pmc-child --steps 2 --warmup 1 "$@" > $OUT/ch_$name.log 2>&1
  local rc=$?; echo "ch $name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/ch_$name.log; exit $rc; }
}
ALL=$(python3 -c "print(' '.join(f'AQZ_RDREQ_CH{k}' for k in range(16)))")
run probe2 "AQZ_RDREQ_CH0 AQZ_RDREQ_CH1" --workload 1024x1024x256_u16 --method decimate
run v1024_dec "$ALL" --workload 1024x1024x256_u16 --method decimate
run v1024_mean "$ALL" --workload 1024x1024x256_u16 --method mean
run v512_dec "$ALL" --workload 1024x1024x256_u16 --method decimate --shape 512x512
run v2048_dec "$ALL" --workload 1024x1024x256_u16 --method decimate --shape 2048x2048
run v4096_dec "$ALL" --workload 1024x1024x256_u16 --method decimate --shape 4096x4096
python3 scripts/channel_table.py $OUT
echo "== done"
