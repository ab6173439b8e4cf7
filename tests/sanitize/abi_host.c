/* ASan/UBSan exercise of the product library's host-only entry points
 * (planner, argument validation, method strings) — no GPU needed.
 * Built and run by scripts/sanitize.sh against a host-sanitized build of
 * libaqz_downsampler. */
#include "aqz_blosc.h"
#include "aqz_downsampler.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int
main(void)
{
    aqz_dimension d[5] = { { AQZ_DIM_TIME, 0, 5, 1, 1.0 },
                           { AQZ_DIM_CHANNEL, 3, 1, 3, 1.0 },
                           { AQZ_DIM_SPACE, 128, 8, 1, 1.0 },
                           { AQZ_DIM_SPACE, 512, 64, 1, 1.0 },
                           { AQZ_DIM_SPACE, 512, 64, 1, 1.0 } };
    uint32_t n = 0;
    if (aqz_plan_levels(d, 5, 0, NULL, 0, &n) || n != 5)
        return 1;
    aqz_dimension out[25];
    if (aqz_plan_levels(d, 5, 0, out, 2, &n) != AQZ_OVERFLOW)
        return 2;
    if (aqz_plan_levels(d, 5, 0, out, 5, &n) || out[4 * 5 + 2].array_size_px != 8)
        return 3;
    if (aqz_plan_levels(d, 2, 0, out, 5, &n) != AQZ_INVALID_ARGUMENT)
        return 4;
    if (strlen(aqz_last_error()) == 0)
        return 5;
    aqz_level_desc lv[3] = { { 64, 48, 1 }, { 32, 24, 1 }, { 16, 12, 1 } };
    aqz_ds* ds = NULL;
    if (aqz_ds_create(lv, 3, 99, 1, 0, &ds) != AQZ_INVALID_ARGUMENT || ds)
        return 6;
    if (aqz_ds_create(lv, 3, 1, 7, 0, &ds) != AQZ_INVALID_ARGUMENT || ds)
        return 7;
    aqz_level_desc bad[2] = { { 64, 48, 1 }, { 30, 24, 1 } };
    if (aqz_ds_create(bad, 2, 1, 1, 0, &ds) != AQZ_INVALID_ARGUMENT || ds)
        return 8;
    if (aqz_ds_create(lv, 0, 1, 1, 0, &ds) != AQZ_INVALID_ARGUMENT)
        return 9;
    for (int m = -1; m < 5; ++m) {
        const char* nm = aqz_method_name(m);
        const char* js = aqz_method_metadata_json(m);
        if ((m >= 0 && m < 4) != (nm != NULL && js != NULL))
            return 10;
    }
    int has = 1;
    if (aqz_ds_take_frame(NULL, 1, NULL, 0, NULL, &has) != AQZ_INVALID_ARGUMENT)
        return 11;
    /* round-2 entry points: null handles are rejected without touching memory */
    uint32_t tr[3] = { 0, 256, 256 }, tc[3] = { 0, 256, 256 };
    void* outs[3] = { NULL, NULL, NULL };
    if (aqz_ds_run_device_batch_tiled(NULL, NULL, 1, tr, tc, outs, NULL, NULL, NULL) !=
        AQZ_INVALID_ARGUMENT)
        return 12;
    if (aqz_ds_tiled_flag_slots(NULL, 1, 256, 256) != 0)
        return 13;
    if (aqz_ds_run_device_batch(NULL, NULL, 1, outs, NULL, NULL) != AQZ_INVALID_ARGUMENT)
        return 14;
    aqz_ds_destroy(NULL);
    if (aqz_ds_run_device_batch_chunked(NULL, NULL, 1, NULL, NULL, NULL, NULL) !=
        AQZ_INVALID_ARGUMENT)
        return 15;
    /* chunk-lattice offsets (T/C/Y/X, ragged chunks) */
    aqz_dimension nd[4] = { { AQZ_DIM_TIME, 0, 2, 1, 1.0 },
                            { AQZ_DIM_CHANNEL, 3, 2, 1, 1.0 },
                            { AQZ_DIM_SPACE, 100, 32, 1, 1.0 },
                            { AQZ_DIM_SPACE, 90, 64, 1, 1.0 } };
    uint64_t offs[37], cb = 0, lb = 0;
    if (aqz_chunk_frame_offsets(nd, 4, 2, 5, 37, offs, &cb, &lb) ||
        cb != 2ull * 2 * 2 * 32 * 64 || lb != 2 * 4 * 2 * cb)
        return 16;
    if (aqz_chunk_frame_offsets(nd, 2, 2, 0, 1, offs, &cb, &lb) != AQZ_INVALID_ARGUMENT)
        return 17;
    /* blosc frames from host-filtered blocks: every destination size from
     * too small to roomy, compressible and incompressible chunks, both codecs;
     * with byte shuffle off the "filtered" bytes are the chunk itself */
    const size_t nb = 70001;
    uint8_t* src = (uint8_t*)malloc(nb);
    uint32_t x = 1;
    for (size_t i = 0; i < nb; ++i) {
        x = x * 1664525u + 1013904223u;
        src[i] = (uint8_t)(i < nb / 2 ? (i / 97) & 7 : x >> 24);
    }
    const char* codecs[2] = { "lz4", "zstd" };
    for (int c = 0; c < 2; ++c)
        for (int clevel = 0; clevel <= 9; clevel += 3)
            for (size_t dsz = 10; dsz < nb + 200; dsz += 7001) {
                uint8_t* dst = (uint8_t*)malloc(dsz);
                size_t fb = 0;
                int raw = 0;
                uint32_t bs = 0;
                if (aqz_blosc_blocksize(clevel, 1, nb, codecs[c], &bs) || bs == 0)
                    return 18;
                if (aqz_blosc_frame_from_filtered(clevel, 0, 1, codecs[c], src, src, nb, dst,
                                                  dsz, &fb, &raw))
                    return 19;
                if (fb > dsz)
                    return 20;
                free(dst);
            }
    uint32_t bs = 0;
    if (aqz_blosc_blocksize(10, 2, nb, "lz4", &bs) != AQZ_INVALID_ARGUMENT ||
        aqz_blosc_blocksize(5, 2, nb, "blosclz", &bs) != AQZ_INVALID_ARGUMENT)
        return 21;
    free(src);
    /* node sharding: shard units (host only) and create-time validation */
    {
        aqz_level_desc vol[3] = { { 64, 64, 16 }, { 32, 32, 8 }, { 16, 16, 4 } };
        aqz_level_desc odd[3] = { { 64, 64, 15 }, { 32, 32, 8 }, { 16, 16, 4 } };
        aqz_level_desc flat[2] = { { 64, 64, 0 }, { 32, 32, 0 } };
        uint32_t unit = 0, per[3] = { 0 };
        if (aqz_shard_unit(vol, 3, &unit, per) || unit != 4 || per[1] != 2 || per[2] != 1)
            return 22;
        if (aqz_shard_unit(odd, 3, &unit, per) || unit != 15 || per[1] != 8 || per[2] != 4)
            return 23;
        if (aqz_shard_unit(flat, 2, &unit, NULL) || unit != 1)
            return 24;
        if (aqz_shard_unit(NULL, 3, &unit, per) != AQZ_INVALID_ARGUMENT)
            return 25;
        int devs[2] = { 0, 0 };
        aqz_node* node = NULL;
        if (aqz_node_create(vol, 3, 10, 1, devs, 2, &node) != AQZ_INVALID_ARGUMENT || node)
            return 26;
        if (aqz_node_create(vol, 3, 1, 1, devs, 0, &node) != AQZ_INVALID_ARGUMENT || node)
            return 27;
        aqz_node_destroy(NULL);
        int has = 1;
        if (aqz_node_add_frame(NULL, devs, 4) != AQZ_INVALID_ARGUMENT ||
            aqz_node_take_frame(NULL, 1, NULL, 0, NULL, &has) != AQZ_INVALID_ARGUMENT ||
            aqz_node_flush(NULL) != AQZ_INVALID_ARGUMENT)
            return 28;
        int done = 0;
        if (aqz_ds_poll(NULL, &done) != AQZ_INVALID_ARGUMENT)
            return 29;
        /* round-5 entry points: NULL handles refused, nothing touched */
        uint32_t counts[3] = { 0 };
        void* outs[3] = { NULL, NULL, NULL };
        if (aqz_node_run_device_batch(NULL, devs, 0, 4, outs, counts, NULL, 0) !=
              AQZ_INVALID_ARGUMENT ||
            aqz_node_set_level_tiling(NULL, 1, 16, 16) != AQZ_INVALID_ARGUMENT ||
            aqz_node_wait_input(NULL) != AQZ_INVALID_ARGUMENT ||
            aqz_ds_wait_input(NULL) != AQZ_INVALID_ARGUMENT)
            return 30;
    }
    printf("abi_host: ok (%s; %s)\n", aqz_version(), aqz_blosc_codec_info());
    return 0;
}
