#!/bin/bash
# Round 6: counter evidence for V Decimate's read rate.
#  * per-channel TCC read requests (tools/pmc/tcc_channels.yaml) of
#    volume_kernel<u16, Decimate>: one volume, four volumes (ZFAST order),
#    and V Mean (dense rows, same kernel);
#  * read latency and DRAM credit stalls (TCC_EA0_RDREQ_LEVEL / RDREQ:
#    requests in flight per request = mean cycles a read waits, Little's law)
#    for the same launches, the headline, and the dense-row / Decimate-row
#    probe (tools/pitch_probe.py --set volume).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r06_vdec_pmc; mkdir -p $OUT
export TMPDIR=/tmp
Y=$PWD/tools/pmc/tcc_channels.yaml
ALL=$(python3 -c "print(' '.join(f'AQZ_RDREQ_CH{k}' for k in range(16)))")
LAT="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum"
run() { # name "counters" extra-rocprof-args -- command...
  local name=$1 ctrs=$2; shift 2
  rm -rf $OUT/$name
  timeout -s KILL 120 rocprofv3 -E $Y --pmc $ctrs --output-format csv -d $OUT/$name -o run -- \
    "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/$name.log; exit $rc; }
}
V="python3 bench.py --pmc-child --steps 2 --warmup 1 --workload 1024x1024x256_u16"
run ch_v4_dec "$ALL" $V --method decimate
run ch_v1_dec "$ALL" $V --method decimate --batch 256
run ch_v4_mean "$ALL" $V --method mean
run lat_v4_dec "$LAT" $V --method decimate
run lat_v1_dec "$LAT" $V --method decimate --batch 256
run lat_v4_mean "$LAT" $V --method mean
run lat_headline "$LAT" python3 bench.py --pmc-child --steps 2 --warmup 1
run lat_probe "$LAT" python3 tools/pitch_probe.py --set volume --reps 3
python3 scripts/pmc_latency.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
echo "== done"
