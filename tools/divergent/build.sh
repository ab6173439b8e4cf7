#!/bin/bash
# Regression probe for the round-5 lane-divergent NaN fix-up (VERDICT r5 #1,
# docs/HISTORY.md §11.6): builds variant copies of libaqz_downsampler.so whose
# shard 0 (u8 + f32 kernels) is compiled with -DAQZ_NAN_FIXUP_DIVERGENT=1,
# each with one extra compiler option, into tools/divergent/lib_<name>.so.
# The other objects are the product build's (make -C acquire-zarr_amd first).
#   ./tools/divergent/build.sh div "" divsel "-DAQZ_EDGE_LOAD_SELECT=1"
# div = round 5's form (divergent branch + the product's exec-masked edge
# loads), divsel = the divergent branch over edge loads issued on every lane
# (DESIGN.md §12.1).
# RELINK=1 keeps an existing variant shard object and only relinks it against
# the current product objects (after C-ABI changes).
# Not product code: only tests/test_gpu_divergent.py and tests/narrow_dbg.py
# load these libraries (via $AQZ_LIB_PATH).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
B=$ROOT/acquire-zarr_amd/build
HIPFLAGS="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -Wall -Wno-unused-function"
INC="-I$ROOT/include -I$ROOT/acquire-zarr_amd/csrc"
# DIVERGENT=0 builds the product's (wave-uniform) form with the extra options
DIVFLAG="-DAQZ_NAN_FIXUP_DIVERGENT=1"
[ "${DIVERGENT:-1}" = 0 ] && DIVFLAG=""
# SHARD=k: vary dtype shard k instead of 0 (1 holds the u16 kernels)
SHARD=${SHARD:-0}
pids=()
names=()
while [ $# -ge 2 ]; do
  name=$1; extra=$2; shift 2
  mkdir -p "$ROOT/tools/divergent/build_$name"
  (
    if [ "${RELINK:-0}" != 1 ] || [ ! -f "$ROOT/tools/divergent/build_$name/ds_kernels_s$SHARD.o" ]; then
      /opt/rocm/bin/hipcc $HIPFLAGS $INC -DAQZ_SHARDS=8 -DAQZ_SHARD=$SHARD $DIVFLAG $extra \
        -c "$ROOT/acquire-zarr_amd/csrc/ds_kernels.hip" -o "$ROOT/tools/divergent/build_$name/ds_kernels_s$SHARD.o"
    fi
    objs=("$ROOT/tools/divergent/build_$name/ds_kernels_s$SHARD.o")
    for o in "$B"/*.o; do
      [ "$(basename "$o")" = ds_kernels_s$SHARD.o ] || objs+=("$o")
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/divergent/lib_$name.so" \
      "${objs[@]}" -Wl,-rpath,/opt/rocm/lib -ldl -lpthread
  ) > "$ROOT/tools/divergent/build_$name.log" 2>&1 &
  pids+=($!)
  names+=("$name")
done
rc=0
for i in "${!pids[@]}"; do
  if wait "${pids[$i]}"; then echo "built lib_${names[$i]}.so"; else echo "FAILED ${names[$i]}"; rc=1; fi
done
exit $rc
