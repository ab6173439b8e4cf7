#!/bin/bash
# Closing check of the final tree: the default bench line, and the
# rocprofv3 kernel-trace summary of the same command.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/r04_closing
mkdir -p $out
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o headline -- \
  python $GRAFT_REPO_ROOT/bench.py --no-pmc --cpu-seconds 0 --e2e-frames 0 > $out/prof_bench.json 2> $out/prof.err
