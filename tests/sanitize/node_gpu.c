/*
 * Host-code AddressSanitizer/UBSan run of the library's node paths ON the GPU
 * (scripts/sanitize_gpu_build.sh, scripts/r05_sanitize_gpu.sh): the library's host code (ds_runtime.cpp,
 * ds_node.cpp, ...) is built with -Xarch_host -fsanitize=address,undefined,
 * its kernels are plain gfx950 code.  Small 2-D and volume pyramids go
 * through one handle (the expected bytes) and through aqz_node on handles
 * that repeat device 0: the host batch, the device batch in place and staged
 * (AQZ_NODE_STAGE_ALL: peer-copy staging, three streams and events), the
 * stream (add / wait_input / take / flush), the stream as the drop-in's
 * node mode runs it (buffers kept until aqz_node_inputs_released counts
 * them; round 6), and the single-handle async add with
 * aqz_ds_input_pending.  Every result is compared byte for byte with the
 * one-handle run.  Exits nonzero on the first mismatch or error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "aqz_downsampler.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_ != 0) {                                                            \
            fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, rc_);     \
            return 1;                                                              \
        }                                                                          \
    } while (0)
#define HIPCHECK(x) CHECK((int)(x))

enum { MAXL = 4 };

static uint32_t lcg(uint32_t* s) { *s = *s * 1664525u + 1013904223u; return *s >> 8; }

static size_t level_bytes(const aqz_level_desc* l) { return (size_t)l->width * l->height * 2; }

/* one pyramid: levels, frame count; returns 0 when every path agrees */
static int
run_case(const aqz_level_desc* lv, uint32_t nl, uint32_t n, int method, const char* name)
{
    const size_t fb = level_bytes(&lv[0]);
    uint8_t* host = malloc(fb * n);
    uint32_t seed = 12345u + n;
    for (size_t i = 0; i < fb * n; ++i)
        host[i] = (uint8_t)lcg(&seed);

    /* expected: one handle, device batch */
    aqz_ds* ds = NULL;
    CHECK(aqz_ds_create(lv, nl, AQZ_DTYPE_UINT16, method, 0, &ds));
    void* d_in = NULL;
    HIPCHECK(hipMalloc(&d_in, fb * n));
    HIPCHECK(hipMemcpy(d_in, host, fb * n, hipMemcpyHostToDevice));
    void* d_ref[MAXL] = { 0 };
    void* d_out[MAXL] = { 0 };
    uint8_t* ref[MAXL] = { 0 };
    uint8_t* got[MAXL] = { 0 };
    uint32_t cref[MAXL] = { 0 }, cgot[MAXL] = { 0 };
    for (uint32_t L = 1; L < nl; ++L) {
        const size_t cap = level_bytes(&lv[L]) * n;
        HIPCHECK(hipMalloc(&d_ref[L], cap));
        HIPCHECK(hipMalloc(&d_out[L], cap));
        ref[L] = calloc(1, cap);
        got[L] = calloc(1, cap);
    }
    CHECK(aqz_ds_run_device_batch(ds, d_in, n, d_ref, cref, NULL));
    HIPCHECK(hipDeviceSynchronize());
    for (uint32_t L = 1; L < nl; ++L)
        HIPCHECK(hipMemcpy(ref[L], d_ref[L], level_bytes(&lv[L]) * cref[L], hipMemcpyDeviceToHost));
    aqz_ds_destroy(ds);

    const int devs[3] = { 0, 0, 0 };
    aqz_node* node = NULL;
    CHECK(aqz_node_create(lv, nl, AQZ_DTYPE_UINT16, method, devs, 3, &node));

    /* node device batch: in place, then staged through the handles' buffers */
    for (int staged = 0; staged < 2; ++staged) {
        for (uint32_t L = 1; L < nl; ++L)
            HIPCHECK(hipMemset(d_out[L], 0xA5, level_bytes(&lv[L]) * n));
        CHECK(aqz_node_run_device_batch(node, d_in, 0, n, d_out, cgot, NULL,
                                        staged ? AQZ_NODE_STAGE_ALL : 0u));
        HIPCHECK(hipDeviceSynchronize());
        for (uint32_t L = 1; L < nl; ++L) {
            const size_t nb = level_bytes(&lv[L]) * cref[L];
            if (cgot[L] != cref[L])
                return fprintf(stderr, "%s device batch staged=%d L%u count %u != %u\n", name,
                               staged, L, cgot[L], cref[L]), 1;
            HIPCHECK(hipMemcpy(got[L], d_out[L], nb, hipMemcpyDeviceToHost));
            if (memcmp(got[L], ref[L], nb))
                return fprintf(stderr, "%s device batch staged=%d L%u differs\n", name, staged,
                               L), 1;
        }
    }

    /* node host batch */
    void* houts[MAXL] = { 0 };
    for (uint32_t L = 1; L < nl; ++L) {
        memset(got[L], 0, level_bytes(&lv[L]) * n);
        houts[L] = got[L];
    }
    CHECK(aqz_node_run_host_batch(node, host, n, houts, cgot));
    for (uint32_t L = 1; L < nl; ++L)
        if (cgot[L] != cref[L] || memcmp(got[L], ref[L], level_bytes(&lv[L]) * cref[L]))
            return fprintf(stderr, "%s host batch L%u differs\n", name, L), 1;

    /* node stream: add, wait_input (the frame may be reused), take whatever is
     * ready, flush, drain; the frames are copied into one reused buffer to
     * show wait_input's contract */
    uint8_t* slot = malloc(fb);
    size_t taken[MAXL] = { 0 };
    for (uint32_t k = 0; k <= n; ++k) {
        if (k < n) {
            memcpy(slot, host + fb * k, fb);
            CHECK(aqz_node_add_frame(node, slot, fb));
            CHECK(aqz_node_wait_input(node));
        } else {
            CHECK(aqz_node_flush(node));
        }
        for (uint32_t L = 1; L < nl; ++L) {
            for (;;) {
                const size_t lb = level_bytes(&lv[L]);
                size_t nb = 0;
                int has = 0;
                if (taken[L] >= cref[L])
                    break;
                CHECK(aqz_node_take_frame(node, L, got[L] + taken[L] * lb, lb, &nb, &has));
                if (!has)
                    break;
                if (nb != lb)
                    return fprintf(stderr, "%s stream L%u nbytes %zu\n", name, L, nb), 1;
                ++taken[L];
            }
        }
    }
    free(slot);
    for (uint32_t L = 1; L < nl; ++L)
        if (taken[L] != cref[L] || memcmp(got[L], ref[L], level_bytes(&lv[L]) * cref[L]))
            return fprintf(stderr, "%s stream L%u differs (%zu frames)\n", name, L, taken[L]), 1;

    /* node stream as the drop-in's node mode runs it (round 6,
     * Downsampler::release_frame): no wait_input; a frame's buffer is kept
     * until aqz_node_inputs_released counts the frame, then rewritten with a
     * later one (three buffers for three handles) */
    {
        enum { NB = 3 };
        uint8_t* bufs[NB];
        uint64_t holds[NB]; /* frame id the buffer was given, or UINT64_MAX */
        uint64_t base = 0, released = 0;
        CHECK(aqz_node_inputs_released(node, &base)); /* every earlier frame */
        for (int b = 0; b < NB; ++b) {
            bufs[b] = malloc(fb);
            holds[b] = UINT64_MAX;
        }
        memset(taken, 0, sizeof taken);
        for (uint32_t k = 0; k <= n; ++k) {
            if (k < n) {
                int b = -1;
                for (long spin = 0; b < 0 && spin < 2000000; ++spin) {
                    CHECK(aqz_node_inputs_released(node, &released));
                    for (int i = 0; i < NB && b < 0; ++i)
                        if (holds[i] == UINT64_MAX || holds[i] < released)
                            b = i;
                }
                if (b < 0)
                    return fprintf(stderr, "%s keep: no buffer released\n", name), 1;
                memcpy(bufs[b], host + fb * k, fb);
                CHECK(aqz_node_add_frame(node, bufs[b], fb));
                holds[b] = base + k;
            } else {
                CHECK(aqz_node_flush(node));
            }
            for (uint32_t L = 1; L < nl; ++L) {
                for (;;) {
                    const size_t lb = level_bytes(&lv[L]);
                    size_t nb = 0;
                    int has = 0;
                    if (taken[L] >= cref[L])
                        break;
                    CHECK(aqz_node_take_frame(node, L, got[L] + taken[L] * lb, lb, &nb, &has));
                    if (!has)
                        break;
                    ++taken[L];
                }
            }
        }
        CHECK(aqz_node_inputs_released(node, &released));
        if (released != base + n)
            return fprintf(stderr, "%s keep: released %llu of %llu\n", name,
                           (unsigned long long)released, (unsigned long long)(base + n)), 1;
        for (int b = 0; b < NB; ++b)
            free(bufs[b]);
        for (uint32_t L = 1; L < nl; ++L)
            if (taken[L] != cref[L] || memcmp(got[L], ref[L], level_bytes(&lv[L]) * cref[L]))
                return fprintf(stderr, "%s keep L%u differs (%zu frames)\n", name, L, taken[L]), 1;
    }
    aqz_node_destroy(node);

    /* single handle, async add + wait_input + take */
    CHECK(aqz_ds_create(lv, nl, AQZ_DTYPE_UINT16, method, 0, &ds));
    size_t taken1[MAXL] = { 0 };
    for (uint32_t k = 0; k < n; ++k) {
        CHECK(aqz_ds_add_frame_async(ds, host + fb * k, fb));
        int pend = -1;
        CHECK(aqz_ds_input_pending(ds, &pend)); /* 0 or 1, either is right here */
        if (pend != 0 && pend != 1)
            return fprintf(stderr, "%s input_pending %d\n", name, pend), 1;
        CHECK(aqz_ds_wait_input(ds));
        CHECK(aqz_ds_input_pending(ds, &pend));
        if (pend != 0)
            return fprintf(stderr, "%s input still pending after wait_input\n", name), 1;
        CHECK(aqz_ds_wait(ds));
        for (uint32_t L = 1; L < nl; ++L) {
            const size_t lb = level_bytes(&lv[L]);
            size_t nb = 0;
            int has = 0;
            if (taken1[L] >= cref[L])
                continue;
            CHECK(aqz_ds_take_frame(ds, L, got[L] + taken1[L] * lb, lb, &nb, &has));
            if (has)
                ++taken1[L];
        }
    }
    for (uint32_t L = 1; L < nl; ++L)
        if (taken1[L] != cref[L] || memcmp(got[L], ref[L], level_bytes(&lv[L]) * cref[L]))
            return fprintf(stderr, "%s async L%u differs (%zu frames)\n", name, L, taken1[L]), 1;
    aqz_ds_destroy(ds);

    for (uint32_t L = 1; L < nl; ++L) {
        HIPCHECK(hipFree(d_ref[L]));
        HIPCHECK(hipFree(d_out[L]));
        free(ref[L]);
        free(got[L]);
    }
    HIPCHECK(hipFree(d_in));
    free(host);
    printf("node_gpu: %s ok (%u frames, %u levels)\n", name, n, nl);
    return 0;
}

int
main(void)
{
    setvbuf(stdout, NULL, _IONBF, 0); /* LSan's exit path skips stdio flushing */
    const aqz_level_desc flat[3] = { { 256, 192, 0 }, { 128, 96, 0 }, { 64, 48, 0 } };
    const aqz_level_desc vol[3] = { { 128, 96, 16 }, { 64, 48, 8 }, { 32, 24, 4 } };
    /* $AQZ_SAN_REPEAT rounds of every case: a leak in the library grows with
     * it, the runtimes' one-off allocations do not */
    const char* rep = getenv("AQZ_SAN_REPEAT");
    const int rounds = rep && atoi(rep) > 0 ? atoi(rep) : 1;
    for (int r = 0; r < rounds; ++r)
        if (run_case(flat, 3, 9, AQZ_METHOD_MEAN, "2-D mean") ||
            run_case(flat, 3, 7, AQZ_METHOD_MAX, "2-D max") ||
            run_case(vol, 3, 16, AQZ_METHOD_MEAN, "volume mean") ||
            run_case(vol, 3, 16, AQZ_METHOD_DECIMATE, "volume decimate"))
            return 1;
    printf("node_gpu: all clean (%s)\n", aqz_version());
    return 0;
}
