/* ASan/UBSan exercise of the C oracle (host code only): every dtype x method
 * through scale_image, average_two_frames, the planner, the add/take state
 * machine and chunk tiling, on random sizes including 1x1 and odd edges.
 * Built and run by scripts/sanitize.sh. */
#include "../../oracle/ds_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t
next(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

static void
fill(uint8_t* p, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        p[i] = (uint8_t)next();
}

int
main(void)
{
    for (int iter = 0; iter < 400; ++iter) {
        const int dt = (int)(next() % 10), m = (int)(next() % 4);
        const size_t bpp = oracle_bytes_of_type(dt);
        const uint32_t w = 1 + next() % 97, h = 1 + next() % 61;
        uint8_t* img = malloc(w * h * bpp);
        fill(img, w * h * bpp);
        uint8_t* out = malloc(((w + 1) / 2) * ((h + 1) / 2) * bpp);
        if (oracle_scale_image(dt, m, img, w, h, out))
            return 1;
        uint8_t* twin = malloc(w * h * bpp);
        fill(twin, w * h * bpp);
        if (oracle_average_two_frames(dt, m, img, twin, (size_t)w * h))
            return 1;
        const uint32_t tr = 1 + next() % 17, tc = 1 + next() % 33;
        const uint32_t nt = ((w + tc - 1) / tc) * ((h + tr - 1) / tr);
        uint8_t* tiles = malloc((size_t)nt * tr * tc * bpp);
        uint8_t* nz = malloc(nt);
        if (oracle_tile_frame(dt, img, w, h, tr, tc, tiles, nz))
            return 1;
        free(tiles);
        free(nz);
        free(twin);
        free(out);
        free(img);
    }
    /* planner + state machine on random 3..5-D configurations */
    for (int iter = 0; iter < 300; ++iter) {
        oracle_dim dims[5];
        const uint32_t nd = 3 + next() % 3;
        for (uint32_t i = 0; i < nd; ++i) {
            dims[i].type = i + 2 < nd ? (int)(next() % 4) : 0;
            dims[i].array_size_px = 1 + next() % 70;
            dims[i].chunk_size_px = 1 + next() % 20;
            dims[i].shard_size_chunks = 1 + next() % 4;
            dims[i].scale = 1.0;
        }
        /* size query with a cap, then the capped plan into an exact buffer,
         * then a too-small buffer (must fail cleanly), then the full plan */
        const uint32_t cap = next() % 4;
        uint32_t n = 0;
        if (oracle_plan_levels(dims, nd, cap, NULL, 0, &n))
            return 1;
        oracle_dim* capped = malloc(sizeof(oracle_dim) * nd * n);
        if (oracle_plan_levels(dims, nd, cap, capped, n, &n))
            return 1;
        if (n > 1 && oracle_plan_levels(dims, nd, cap, capped, n - 1, &n) != -2)
            return 1;
        free(capped);
        uint32_t n2 = 0;
        if (oracle_plan_levels(dims, nd, 0, NULL, 0, &n2))
            return 1;
        oracle_dim* lv = malloc(sizeof(oracle_dim) * nd * n2);
        if (oracle_plan_levels(dims, nd, 0, lv, n2, &n2))
            return 1;
        uint32_t W[32], H[32], P[32];
        for (uint32_t l = 0; l < n2; ++l) {
            W[l] = lv[l * nd + nd - 1].array_size_px;
            H[l] = lv[l * nd + nd - 2].array_size_px;
            P[l] = lv[l * nd + nd - 3].array_size_px;
        }
        const int dt = (int)(next() % 10), m = (int)(next() % 4);
        oracle_ds* ds = oracle_ds_create(W, H, P, n2, dt, m);
        if (!ds)
            return 1;
        const size_t fb = (size_t)W[0] * H[0] * oracle_bytes_of_type(dt);
        uint8_t* frame = malloc(fb);
        uint8_t* dst = malloc(fb);
        for (int f = 0; f < 9; ++f) {
            fill(frame, fb);
            if (oracle_ds_add_frame(ds, frame, fb))
                return 1;
            for (uint32_t l = 1; l < n2; ++l)
                if (next() % 3)
                    oracle_ds_take_frame(ds, l, dst, fb, NULL);
        }
        oracle_ds_destroy(ds);
        free(dst);
        free(frame);
        free(lv);
    }
    printf("oracle_fuzz: ok\n");
    return 0;
}
