#!/bin/bash
# Host-code sanitizers (GPU ASan is not available on this pool):
#  1. the C oracle under ASan+UBSan (gcc), driven by tests/sanitize/oracle_fuzz.c
#  2. the product library's host code under ASan+UBSan (hipcc -Xarch_host),
#     driven by tests/sanitize/abi_host.c (planner, validation, strings,
#     chunk-lattice offsets, the blosc frame writer with real LZ4/zstd).
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${TMPDIR:-/tmp}/aqz_sanitize"
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer"
gcc -O1 -g $SAN -std=c11 -I"$ROOT/oracle" "$ROOT/tests/sanitize/oracle_fuzz.c" \
    "$ROOT/oracle/ds_oracle.c" -o "$OUT/oracle_fuzz"
"$OUT/oracle_fuzz"
HIPCC=/opt/rocm/bin/hipcc
HF="-O1 -g -std=c++20 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$ROOT/acquire-zarr_amd/csrc"
HS="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
# ds_kernels.hip in the library's 8 dtype shards, in parallel (ds_dispatch.cpp
# routes the launchers), like acquire-zarr_amd/Makefile
pids=()
for k in 0 1 2 3 4 5 6 7; do
  $HIPCC $HF $HS -DAQZ_SHARDS=8 -DAQZ_SHARD=$k -x hip -c "$ROOT/acquire-zarr_amd/csrc/ds_kernels.hip" \
      -o "$OUT/ds_kernels_s$k.o" &
  pids+=($!)
done
for f in ds_dispatch.cpp ds_runtime.cpp ds_node.cpp codec_runtime.cpp blosc_frame.cpp; do
  $HIPCC $HF $HS -DAQZ_SHARDS=8 -x hip -c "$ROOT/acquire-zarr_amd/csrc/$f" -o "$OUT/${f%.*}.o"
done
$HIPCC $HF $HS -c "$ROOT/acquire-zarr_amd/csrc/codec_kernels.hip" -o "$OUT/codec_kernels.o"
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -fsanitize=address,undefined \
    "$OUT"/ds_kernels_s?.o "$OUT/ds_dispatch.o" "$OUT/ds_runtime.o" "$OUT/ds_node.o" "$OUT/codec_runtime.o" \
    "$OUT/codec_kernels.o" "$OUT/blosc_frame.o" -o "$OUT/libaqz_san.so" \
    -Wl,-rpath,/opt/rocm/lib -ldl -lpthread
# the driver must use the same (clang) sanitizer runtime as the library
/opt/rocm/lib/llvm/bin/clang -g -fsanitize=address,undefined -I"$ROOT/include" \
    "$ROOT/tests/sanitize/abi_host.c" "$OUT/libaqz_san.so" \
    -Wl,-rpath,"$OUT" -Wl,-rpath,/opt/rocm/lib -o "$OUT/abi_host"
ASAN_OPTIONS=detect_leaks=1 "$OUT/abi_host"
echo "sanitize: all clean"
