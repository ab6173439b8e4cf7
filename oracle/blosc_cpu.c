/*
 * blosc_cpu.c — CPU BASELINE (bench infrastructure only): the reference's
 * chunk compression as it runs, from C threads.
 *
 * The reference compresses each chunk with
 *   blosc_compress_ctx(clevel, shuffle, typesize, nbytes, src, dest,
 *                      nbytes + 16, cname, 0, 1)
 * (zarr.common.cpp:106-137), one job per chunk on its thread pool
 * (chunk.cpp:78-105, array.cpp:664-811).  This runs that call on `n_chunks`
 * host chunks spread over `threads` pthreads, using the image's c-blosc
 * (dlopen, $AQZ_LIBBLOSC or /opt/conda/lib/libblosc.so.1), so the baseline
 * has no Python in its loop.  Never linked into the product.
 */
#define _POSIX_C_SOURCE 199309L
#include <dlfcn.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

typedef int (*compress_fn)(int, int, size_t, size_t, const void*, void*, size_t, const char*,
                           size_t, int);

static compress_fn g_compress;

struct job
{
    const uint8_t* src;
    size_t nbytes;
    int n_chunks;
    int clevel, shuffle, typesize;
    const char* cname;
    uint8_t* dst;
    size_t stride;
    size_t* sizes;
    atomic_int next;
    atomic_int failed;
};

static void*
worker(void* arg)
{
    struct job* j = (struct job*)arg;
    for (;;) {
        const int k = atomic_fetch_add(&j->next, 1);
        if (k >= j->n_chunks)
            return NULL;
        const int n = g_compress(j->clevel, j->shuffle, (size_t)j->typesize, j->nbytes,
                                 j->src + (size_t)k * j->nbytes, j->dst + (size_t)k * j->stride,
                                 j->nbytes + 16, j->cname, 0, 1);
        if (n <= 0)
            atomic_store(&j->failed, 1);
        j->sizes[k] = n > 0 ? (size_t)n : 0;
    }
}

static double
now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* Best wall time (s) over `reps` runs; < 0 on error.  dst holds n_chunks
 * frames at `stride` (>= nbytes + 16), sizes their lengths. */
double
cblosc_compress_chunks(const uint8_t* src, size_t nbytes, int n_chunks, int clevel, int shuffle,
                       int typesize, const char* cname, int threads, uint8_t* dst, size_t stride,
                       size_t* sizes, int reps)
{
    if (!g_compress) {
        const char* path = getenv("AQZ_LIBBLOSC");
        void* h = dlopen(path && *path ? path : "/opt/conda/lib/libblosc.so.1", RTLD_NOW);
        if (!h)
            return -1.0;
        g_compress = (compress_fn)dlsym(h, "blosc_compress_ctx");
        if (!g_compress)
            return -1.0;
    }
    if (threads < 1 || threads > 256 || stride < nbytes + 16)
        return -2.0;
    pthread_t tid[256];
    double best = -3.0;
    for (int r = 0; r < reps; ++r) {
        struct job j;
        j.src = src;
        j.nbytes = nbytes;
        j.n_chunks = n_chunks;
        j.clevel = clevel;
        j.shuffle = shuffle;
        j.typesize = typesize;
        j.cname = cname;
        j.dst = dst;
        j.stride = stride;
        j.sizes = sizes;
        atomic_init(&j.next, 0);
        atomic_init(&j.failed, 0);
        const double t0 = now();
        for (int t = 1; t < threads; ++t)
            pthread_create(&tid[t], NULL, worker, &j);
        worker(&j);
        for (int t = 1; t < threads; ++t)
            pthread_join(tid[t], NULL);
        const double dt = now() - t0;
        if (atomic_load(&j.failed))
            return -4.0;
        if (best < 0 || dt < best)
            best = dt;
    }
    return best;
}
