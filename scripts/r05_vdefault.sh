#!/bin/bash
# Round 5: config V at its new default step (four 256-plane volumes): the
# full default line and every method with PMC traffic, data in HBM.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05_vdefault; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload 1024x1024x256_u16 --cpu-seconds 5 > $OUT/v_default.json 2> $OUT/v_default.err || { tail -20 $OUT/v_default.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/v_default.json'));r=d['roofline'];e=d['e2e'];print(d['value'], d['config']['frames_per_step_per_gpu'], r['avg_launch_us'], r['frac'], r['buffer_sets'], r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), r['same_mix_ceiling']['frac_of_ceiling'], d['cpu_baseline']['value'], json.dumps(e.get('node_device_batch'))[:250])"
for m in decimate mean min max; do
  timeout -k 10 300 python bench.py --workload 1024x1024x256_u16 --method $m --steps 20 --warmup 5 --cpu-seconds 0 \
    --e2e-frames 0 > $OUT/m_$m.json 2> $OUT/m_$m.err || { tail -20 $OUT/m_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/m_$m.json'));r=d['roofline'];print('V x4', '$m', d['value'], r['avg_launch_us'], r['frac'], r['buffer_sets'], r.get('same_mix_ceiling',{}).get('frac_of_ceiling'), r['traffic'] and round(r['traffic']/r['alg_bytes_per_launch'],4), d['config']['check'])" | tee -a $OUT/methods.log
done
echo "== done"
