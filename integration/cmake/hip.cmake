# cmake/hip.cmake — multiscale downsampler backend for acquire-zarr, beside
# cmake/simd.cmake and cmake/openmp.cmake (included from the top-level
# CMakeLists.txt right after them; see acquire-zarr-hip.patch).
#
#   AQZ_DOWNSAMPLER=cpu  (default) the reference's SIMD/OpenMP downsampler,
#                        nothing changes.
#   AQZ_DOWNSAMPLER=hip  the per-frame pyramid runs on an MI355X through
#                        libaqz_downsampler (include/aqz_downsampler.h):
#                        src/streaming/downsampler.hip.cpp and array.tiled.cpp
#                        join the target, AQZ_DOWNSAMPLER_HIP selects the
#                        patched code paths, and the library is linked.
#
# AQZ_DS_ROOT points at a built checkout of the MI355X downsampler (the
# directory holding include/aqz_downsampler.h and
# acquire-zarr_amd/libaqz_downsampler.so, built by `make -C acquire-zarr_amd`).

set(AQZ_DOWNSAMPLER "cpu" CACHE STRING
    "Multiscale downsampler backend: cpu (SIMD/OpenMP) or hip (MI355X)")
set_property(CACHE AQZ_DOWNSAMPLER PROPERTY STRINGS cpu hip)
set(AQZ_DS_ROOT "" CACHE PATH
    "MI355X downsampler checkout (include/ and acquire-zarr_amd/libaqz_downsampler.so)")

if (NOT AQZ_DOWNSAMPLER STREQUAL "cpu" AND NOT AQZ_DOWNSAMPLER STREQUAL "hip")
    message(FATAL_ERROR
            "AQZ_DOWNSAMPLER must be 'cpu' or 'hip', got '${AQZ_DOWNSAMPLER}'")
endif ()

function(target_enable_hip_downsampler tgt)
    if (NOT AQZ_DOWNSAMPLER STREQUAL "hip")
        return()
    endif ()

    find_path(AQZ_DS_INCLUDE_DIR aqz_downsampler.h
              HINTS "${AQZ_DS_ROOT}/include"
              REQUIRED)
    find_library(AQZ_DS_LIBRARY aqz_downsampler
                 HINTS "${AQZ_DS_ROOT}/acquire-zarr_amd" "${AQZ_DS_ROOT}/lib"
                 REQUIRED)

    # The adapter sources live next to the target's own (src/streaming).
    target_sources(${tgt} PRIVATE
                   "${CMAKE_CURRENT_SOURCE_DIR}/downsampler.hip.cpp"
                   "${CMAKE_CURRENT_SOURCE_DIR}/array.tiled.cpp")
    target_compile_definitions(${tgt} PRIVATE AQZ_DOWNSAMPLER_HIP)
    target_include_directories(${tgt} PRIVATE "${AQZ_DS_INCLUDE_DIR}")
    target_link_libraries(${tgt} PRIVATE "${AQZ_DS_LIBRARY}")
    message(STATUS "${tgt}: multiscale downsampler on MI355X (${AQZ_DS_LIBRARY})")
endfunction()
