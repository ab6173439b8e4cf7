#!/bin/bash
# Build tests/cpp/bin/adapter_harness: the drop-in zarr::Downsampler as the
# patched reference tree compiles it (AQZ_DOWNSAMPLER_HIP), driven by
# tests/integration/adapter_harness.cpp.  TEST INFRASTRUCTURE.
#
# * a scratch copy of /root/reference (never written to) gets
#   integration/apply.sh; the reference's downsampler.cpp (patched),
#   array.dimensions.cpp, zarr.common.cpp and logger.cpp are compiled from it
#   with the adapter integration/src/streaming/downsampler.hip.cpp;
# * nlohmann/json is the image's genuine 3.1.1 (/opt/conda/include/json.hpp);
#   blosc.h / zstd.h are the image's, and libblosc + its codecs are copied
#   next to the binary (RPATH $ORIGIN/lib) so conda's libstdc++ stays out;
# * linked against acquire-zarr_amd/libaqz_downsampler.so (RPATH relative to
#   the binary, so the built tree runs as-is on the GPU box).
# Needs the reference tree (the build container); the binary travels.
set -euo pipefail
repo="$(cd "$(dirname "$0")/../.." && pwd)"
ref="${AQZ_REFERENCE:-/root/reference}"
out="$repo/tests/cpp/bin"
[ -f "$ref/src/streaming/downsampler.hh" ] || { echo "reference tree absent: $ref" >&2; exit 2; }
[ -f "$repo/acquire-zarr_amd/libaqz_downsampler.so" ] || { echo "build libaqz_downsampler.so first" >&2; exit 2; }
scratch="$(mktemp -d)"
trap 'rm -rf "$scratch"' EXIT
tree="$scratch/acquire-zarr"
mkdir -p "$tree/src"
cp -r "$ref/include" "$ref/cmake" "$tree/"
cp -r "$ref/src/streaming" "$ref/src/logger" "$tree/src/"
cp "$ref/CMakeLists.txt" "$tree/"
"$repo/integration/apply.sh" "$tree" > /dev/null

mkdir -p "$out/lib" "$scratch/inc/nlohmann"
ln -sf /opt/conda/include/json.hpp "$scratch/inc/nlohmann/json.hpp"
for f in libblosc.so.1 liblz4.so.1 libz.so.1 libzstd.so.1; do cp -f "/opt/conda/lib/$f" "$out/lib/$f"; done
ln -sf libblosc.so.1 "$out/lib/libblosc.so"
ln -sf libzstd.so.1 "$out/lib/libzstd.so"

flags=(-std=c++20 -O2 -fPIC -w -DAQZ_DOWNSAMPLER_HIP -I "$scratch/inc" -I "$repo/include"
       -I "$tree/include" -I "$tree/src/streaming" -I "$tree/src/logger" -idirafter /opt/conda/include)
objs=()
pids=()
for s in "$tree/src/streaming/downsampler.cpp" "$tree/src/streaming/downsampler.hip.cpp" \
         "$tree/src/streaming/array.dimensions.cpp" "$tree/src/streaming/zarr.common.cpp" \
         "$tree/src/logger/logger.cpp" "$repo/tests/integration/adapter_harness.cpp"; do
  o="$scratch/$(basename "$s").o"
  g++ "${flags[@]}" -c "$s" -o "$o" &
  pids+=($!)
  objs+=("$o")
done
for p in "${pids[@]}"; do wait "$p"; done
g++ -o "$out/adapter_harness" "${objs[@]}" \
  -L "$repo/acquire-zarr_amd" -laqz_downsampler -L "$out/lib" -lblosc -lzstd -lpthread \
  -Wl,-rpath,'$ORIGIN/../../../acquire-zarr_amd' -Wl,-rpath,'$ORIGIN/lib' -Wl,-rpath,/opt/rocm/lib
echo "built $out/adapter_harness"
