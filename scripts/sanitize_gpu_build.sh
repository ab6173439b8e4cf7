#!/bin/bash
# Host-code ASan/UBSan of the library, run on the GPU (GPU ASan and XNACK are
# not available on this pool; the kernels stay plain gfx950 code, only the
# host code is instrumented).  Builds here, on the CPU:
#   libaqz_san.so (scripts/sanitize.sh objects) + tests/sanitize/bin/node_gpu
# and the GPU box only runs the binary: scripts/r05_sanitize_gpu.sh.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
BIN="$ROOT/tests/sanitize/bin"
SAN_OUT="${TMPDIR:-/tmp}/aqz_sanitize"
[ -f "$SAN_OUT/libaqz_san.so" ] || bash "$ROOT/scripts/sanitize.sh"
mkdir -p "$BIN"
cp "$SAN_OUT/libaqz_san.so" "$BIN/"
/opt/rocm/lib/llvm/bin/clang -g -O1 -fsanitize=address,undefined -fno-omit-frame-pointer \
    -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I"$ROOT/include" \
    "$ROOT/tests/sanitize/node_gpu.c" "$BIN/libaqz_san.so" -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,'$ORIGIN' -Wl,-rpath,/opt/rocm/lib -o "$BIN/node_gpu"
echo "built $BIN/node_gpu"
