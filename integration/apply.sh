#!/bin/bash
# Install the MI355X downsampler backend into an acquire-zarr v0.8.1 source
# tree: copies cmake/hip.cmake and the two new src/streaming sources, then
# applies acquire-zarr-hip.patch (hooks under AQZ_DOWNSAMPLER_HIP only; the
# default AQZ_DOWNSAMPLER=cpu build is unchanged).
#
#   integration/apply.sh <acquire-zarr checkout>
#   cmake -B build -S <checkout> -DAQZ_DOWNSAMPLER=hip -DAQZ_DS_ROOT=<this repo>
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
tree="${1:?usage: apply.sh <acquire-zarr source tree>}"
[ -f "$tree/src/streaming/downsampler.hh" ] || { echo "not an acquire-zarr tree: $tree" >&2; exit 2; }
patch -d "$tree" -p1 --forward --no-backup-if-mismatch < "$here/acquire-zarr-hip.patch"
install -m 0644 "$here/cmake/hip.cmake" "$tree/cmake/hip.cmake"
install -m 0644 "$here/src/streaming/downsampler.hip.cpp" "$tree/src/streaming/downsampler.hip.cpp"
install -m 0644 "$here/src/streaming/array.tiled.cpp" "$tree/src/streaming/array.tiled.cpp"
install -m 0644 "$here/src/streaming/array.tiled.hh" "$tree/src/streaming/array.tiled.hh"
echo "acquire-zarr tree patched: configure with -DAQZ_DOWNSAMPLER=hip -DAQZ_DS_ROOT=$(dirname "$here")"
