#!/bin/bash
# Round 5: float output byte-identical to the reference, NaN payloads
# included — the reference-vector, NaN-vector, adapter,
# parity, tiled and lattice GPU tests, then F (f32) Mean/Max and the headline
# timed to show the NaN fix-up costs nothing measurable.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_nan; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_reference_vectors.py tests/test_gpu_adapter.py tests/test_gpu_parity.py \
  tests/test_gpu_tiled.py tests/test_gpu_lattice.py tests/test_gpu_digests.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for wm in 4096x4096_f32:mean 4096x4096_f32:max 4096x4096_u16:mean; do
  w=${wm%%:*}; m=${wm##*:}
  timeout -k 10 300 python bench.py --workload $w --method $m --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 > $OUT/m_${w}_$m.json 2> $OUT/m_${w}_$m.err || { tail -20 $OUT/m_${w}_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/m_${w}_$m.json'));r=d['roofline'];print('$w', '$m', d['value'], r['avg_launch_us'], r['frac'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/methods.log
done
echo "== done"
