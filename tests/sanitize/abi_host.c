/* ASan/UBSan exercise of the product library's host-only entry points
 * (planner, argument validation, method strings) — no GPU needed.
 * Built and run by scripts/sanitize.sh against a host-sanitized build of
 * libaqz_downsampler. */
#include "aqz_downsampler.h"

#include <stdio.h>
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
    printf("abi_host: ok (%s)\n", aqz_version());
    return 0;
}
