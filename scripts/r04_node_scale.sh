#!/bin/bash
# Rehearse bench.py's N>1 node leg (aqz_node over the ranks' GPUs, run by
# rank 0 while the others wait on a gloo group) on a one-GPU box: two and
# four gloo ranks sharing device 0.
set -e
mkdir -p gpurun_out/r04_node_scale
AQZ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 \
  --cpu-seconds 0 > gpurun_out/r04_node_scale/gpus2.json 2> gpurun_out/r04_node_scale/gpus2.err
AQZ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 5 --warmup 2 \
  --cpu-seconds 0 > gpurun_out/r04_node_scale/gpus4.json 2> gpurun_out/r04_node_scale/gpus4.err
