#!/bin/bash
# Round 5: volume kernel load policy and units per wave.
# Parity first (3-D parity, reference vectors, digests, fuzz), then config V
# under every method with nontemporal loads on and off (AQZ_VOLUME_NT), and
# Decimate with 1 and 2 units per wave (AQZ_VOLUME_UPW), each twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_volume; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_reference_vectors.py tests/test_gpu_digests.py tests/test_gpu_fuzz.py \
  tests/test_gpu_node_device.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # label, env..., then bench args after --
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload 1024x1024x256_u16 --steps 30 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 $BARGS > $OUT/$label.json 2> $OUT/$label.err || { tail -20 $OUT/$label.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$label.json'));r=d['roofline'];print('$label', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/ab.log
}
for rep in 1 2; do
  for m in decimate mean min max; do
    for nt in 1 0; do
      BARGS="--method $m" run ${m}_nt${nt}_r$rep AQZ_VOLUME_NT=$nt
    done
  done
  BARGS="--method decimate" run decimate_nt0_upw1_r$rep AQZ_VOLUME_NT=0 AQZ_VOLUME_UPW=1
done
BARGS="--method decimate" run decimate_default AQZ_UNUSED=0
echo "== done"
