/*
 * ds_oracle.c — CPU ORACLE (test infrastructure only; see ds_oracle.h).
 *
 * Plain-C restatement of acquire-zarr v0.8.1 src/streaming/downsampler.cpp.
 * Each function cites the reference lines it follows.  Scalar and
 * single-threaded on purpose: the reference runs the downsampler on the
 * stream's one frame-queue consumer thread (zarr.stream.cpp:1616-1630) and
 * calls its reducers through a function pointer per output pixel
 * (downsampler.cpp:146-162,198).
 *
 * Arithmetic notes:
 *  - mean4/mean2 are `(a+b+c+d)/4` and `(a+b)/2` under the usual arithmetic
 *    conversions (downsampler.cpp:47-51,108-112).  The "overflow-safe"
 *    integral overloads at :53-62 and :114-123 can never be selected
 *    (`std::enable_if<...>::T` names no member) and are not restated.
 *    Types narrower than int are promoted, so their sums never wrap and the
 *    division truncates toward zero.  32/64-bit sums wrap modulo 2^N; for
 *    the signed types the reference relies on the compiler's two's-complement
 *    wrap (formally UB there) and this file makes that explicit through
 *    unsigned arithmetic.
 *  - float/double sum left to right, ((a+b)+c)+d, then divide by 4.
 *  - min/max are compare-select chains seeded with the first operand
 *    (downsampler.cpp:64-98,125-137), so NaN handling depends on operand
 *    order exactly as in the reference.
 */
#include "ds_oracle.h"

#include <stdlib.h>
#include <string.h>

enum
{
    DT_U8 = 0,
    DT_U16,
    DT_U32,
    DT_U64,
    DT_I8,
    DT_I16,
    DT_I32,
    DT_I64,
    DT_F32,
    DT_F64,
    DT_COUNT
};
enum
{
    M_DECIMATE = 0,
    M_MEAN,
    M_MIN,
    M_MAX,
    M_COUNT
};

size_t
oracle_bytes_of_type(int dtype)
{
    /* zarr.common.cpp:48-69 */
    switch (dtype) {
        case DT_U8:
        case DT_I8:
            return 1;
        case DT_U16:
        case DT_I16:
            return 2;
        case DT_U32:
        case DT_I32:
        case DT_F32:
            return 4;
        case DT_U64:
        case DT_I64:
        case DT_F64:
            return 8;
        default:
            return 0;
    }
}

/* ---- scalar reducers (downsampler.cpp:39-137) ------------------------- */

/* Narrow integers: promoted to int (sum cannot overflow). */
#define MEAN_PROMOTED(T)                                                       \
    static T mean4_##T(T a, T b, T c, T d)                                     \
    {                                                                          \
        return (T)(((int)a + (int)b + (int)c + (int)d) / 4);                   \
    }                                                                          \
    static T mean2_##T(T a, T b) { return (T)(((int)a + (int)b) / 2); }

/* 32/64-bit integers: the sum wraps modulo 2^N, then divides (truncating
 * toward zero for signed types). */
#define MEAN_WRAPPING(T, U)                                                    \
    static T mean4_##T(T a, T b, T c, T d)                                     \
    {                                                                          \
        T s = (T)((U)a + (U)b + (U)c + (U)d);                                  \
        return (T)(s / 4);                                                     \
    }                                                                          \
    static T mean2_##T(T a, T b)                                               \
    {                                                                          \
        T s = (T)((U)a + (U)b);                                                \
        return (T)(s / 2);                                                     \
    }

/* Floating point: left-to-right sum in T, then divide.
 *
 * NaN payloads: C leaves them open, and a compiler may commute `x + y`.  The
 * reference's compiled mean2/mean4 (g++ -O3 -mavx2, oracle/_ref) evaluate
 * `vaddss y, x` with the LEFT operand as the first source, so when both
 * operands are NaN the left one's (quieted) payload survives (Intel SDM
 * vol. 1 table 4-7).  add_<T> pins that order: with two NaNs it returns
 * x + x, whose payload is x's whatever operand order the compiler picks; with
 * one NaN or none the order cannot change the result.  Pinned against the
 * reference by tests/test_reference_pin.py (Z-pair Mean over NaN planes). */
#define MEAN_FLOAT(T)                                                          \
    static T add_##T(T x, T y) { return (x != x && y != y) ? x + x : x + y; }  \
    static T mean4_##T(T a, T b, T c, T d)                                     \
    {                                                                          \
        return add_##T(add_##T(add_##T(a, b), c), d) / 4;                      \
    }                                                                          \
    static T mean2_##T(T a, T b) { return add_##T(a, b) / 2; }

typedef float float32_t;
typedef double float64_t;

MEAN_PROMOTED(uint8_t)
MEAN_PROMOTED(uint16_t)
MEAN_PROMOTED(int8_t)
MEAN_PROMOTED(int16_t)
MEAN_WRAPPING(uint32_t, uint32_t)
MEAN_WRAPPING(uint64_t, uint64_t)
MEAN_WRAPPING(int32_t, uint32_t)
MEAN_WRAPPING(int64_t, uint64_t)
MEAN_FLOAT(float32_t)
MEAN_FLOAT(float64_t)

#define MINMAX(T)                                                              \
    static T min4_##T(T a, T b, T c, T d)                                      \
    {                                                                          \
        T val = a;                                                             \
        if (b < val)                                                           \
            val = b;                                                           \
        if (c < val)                                                           \
            val = c;                                                           \
        if (d < val)                                                           \
            val = d;                                                           \
        return val;                                                            \
    }                                                                          \
    static T max4_##T(T a, T b, T c, T d)                                      \
    {                                                                          \
        T val = a;                                                             \
        if (b > val)                                                           \
            val = b;                                                           \
        if (c > val)                                                           \
            val = c;                                                           \
        if (d > val)                                                           \
            val = d;                                                           \
        return val;                                                            \
    }                                                                          \
    static T min2_##T(T a, T b) { return a < b ? a : b; }                      \
    static T max2_##T(T a, T b) { return a > b ? a : b; }                      \
    static T reduce4_##T(int m, T a, T b, T c, T d)                            \
    {                                                                          \
        switch (m) {                                                           \
            case M_DECIMATE:                                                   \
                return a;                                                      \
            case M_MEAN:                                                       \
                return mean4_##T(a, b, c, d);                                  \
            case M_MIN:                                                        \
                return min4_##T(a, b, c, d);                                   \
            default:                                                           \
                return max4_##T(a, b, c, d);                                   \
        }                                                                      \
    }                                                                          \
    static T reduce2_##T(int m, T a, T b)                                      \
    {                                                                          \
        switch (m) {                                                           \
            case M_DECIMATE:                                                   \
                return a;                                                      \
            case M_MEAN:                                                       \
                return mean2_##T(a, b);                                        \
            case M_MIN:                                                        \
                return min2_##T(a, b);                                         \
            default:                                                           \
                return max2_##T(a, b);                                         \
        }                                                                      \
    }                                                                          \
    /* scale_image<T>, downsampler.cpp:139-206 */                              \
    static void scale_##T(int m, const T* src, size_t width, size_t height,    \
                          T* dst)                                              \
    {                                                                          \
        const size_t w_pad = width + (width % 2);                              \
        const size_t h_pad = height + (height % 2);                            \
        size_t dst_idx = 0;                                                    \
        for (size_t row = 0; row < height; row += 2) {                         \
            const int pad_height = (row == height - 1 && height != h_pad);     \
            for (size_t col = 0; col < width; col += 2) {                      \
                const size_t src_idx = row * width + col;                      \
                const int pad_width = (col == width - 1 && width != w_pad);    \
                T here = src[src_idx];                                         \
                T right = src[src_idx + !pad_width];                           \
                T down = src[src_idx + width * (!pad_height)];                 \
                T diag = src[src_idx + width * (!pad_height) + (!pad_width)];  \
                dst[dst_idx++] = reduce4_##T(m, here, right, down, diag);      \
            }                                                                  \
        }                                                                      \
    }                                                                          \
    /* average_two_frames<T>, downsampler.cpp:208-246 */                       \
    static void avg2_##T(int m, T* dst, const T* src, size_t n)                \
    {                                                                          \
        for (size_t i = 0; i < n; ++i)                                         \
            dst[i] = reduce2_##T(m, dst[i], src[i]);                           \
    }

MINMAX(uint8_t)
MINMAX(uint16_t)
MINMAX(uint32_t)
MINMAX(uint64_t)
MINMAX(int8_t)
MINMAX(int16_t)
MINMAX(int32_t)
MINMAX(int64_t)
MINMAX(float32_t)
MINMAX(float64_t)

#define DISPATCH(dtype, MACRO)                                                 \
    switch (dtype) {                                                           \
        case DT_U8:                                                            \
            MACRO(uint8_t);                                                    \
            break;                                                             \
        case DT_U16:                                                           \
            MACRO(uint16_t);                                                   \
            break;                                                             \
        case DT_U32:                                                           \
            MACRO(uint32_t);                                                   \
            break;                                                             \
        case DT_U64:                                                           \
            MACRO(uint64_t);                                                   \
            break;                                                             \
        case DT_I8:                                                            \
            MACRO(int8_t);                                                     \
            break;                                                             \
        case DT_I16:                                                           \
            MACRO(int16_t);                                                    \
            break;                                                             \
        case DT_I32:                                                           \
            MACRO(int32_t);                                                    \
            break;                                                             \
        case DT_I64:                                                           \
            MACRO(int64_t);                                                    \
            break;                                                             \
        case DT_F32:                                                           \
            MACRO(float32_t);                                                  \
            break;                                                             \
        case DT_F64:                                                           \
            MACRO(float64_t);                                                  \
            break;                                                             \
        default:                                                               \
            return -1;                                                         \
    }

int
oracle_scale_image(int dtype,
                   int method,
                   const void* src,
                   size_t width,
                   size_t height,
                   void* dst)
{
    if (method < 0 || method >= M_COUNT)
        return -1;
#define DO_SCALE(T) scale_##T(method, (const T*)src, width, height, (T*)dst)
    DISPATCH(dtype, DO_SCALE)
#undef DO_SCALE
    return 0;
}

int
oracle_average_two_frames(int dtype,
                          int method,
                          void* dst,
                          const void* src,
                          size_t n_pixels)
{
    if (method < 0 || method >= M_COUNT)
        return -1;
#define DO_AVG(T) avg2_##T(method, (T*)dst, (const T*)src, n_pixels)
    DISPATCH(dtype, DO_AVG)
#undef DO_AVG
    return 0;
}

int
oracle_reduce4(int dtype,
               int method,
               const void* a,
               const void* b,
               const void* c,
               const void* d,
               void* out)
{
    if (method < 0 || method >= M_COUNT)
        return -1;
#define DO_R4(T)                                                               \
    *(T*)out = reduce4_##T(method, *(const T*)a, *(const T*)b, *(const T*)c,  \
                           *(const T*)d)
    DISPATCH(dtype, DO_R4)
#undef DO_R4
    return 0;
}

int
oracle_reduce2(int dtype, int method, const void* a, const void* b, void* out)
{
    if (method < 0 || method >= M_COUNT)
        return -1;
#define DO_R2(T) *(T*)out = reduce2_##T(method, *(const T*)a, *(const T*)b)
    DISPATCH(dtype, DO_R2)
#undef DO_R2
    return 0;
}

/* ---- level planner (downsampler.cpp:8-37, 493-597) -------------------- */

static uint32_t
bit_width_u32(uint32_t x)
{
    uint32_t n = 0;
    while (x) {
        ++n;
        x >>= 1;
    }
    return n;
}

/* downsample_dimension, downsampler.cpp:8-37 */
static oracle_dim
downsample_dimension(oracle_dim dim)
{
    oracle_dim out = dim;
    const uint32_t size = (dim.array_size_px + (dim.array_size_px % 2)) / 2;
    const uint32_t chunk = dim.chunk_size_px;
    const uint32_t n_chunks = (size + chunk - 1) / chunk;
    out.array_size_px = size;
    out.chunk_size_px = chunk;
    out.shard_size_chunks =
      n_chunks < dim.shard_size_chunks ? n_chunks : dim.shard_size_chunks;
    out.scale = dim.scale * 2.0;
    return out;
}

static uint32_t
levels_along(const oracle_dim* d)
{
    const uint32_t n_chunks =
      (d->array_size_px + d->chunk_size_px - 1) / d->chunk_size_px;
    return n_chunks > 1 ? bit_width_u32(n_chunks - 1) : 0;
}

int
oracle_plan_levels(const oracle_dim* dims,
                   uint32_t ndims,
                   uint32_t max_levels,
                   oracle_dim* out,
                   uint32_t out_cap_levels,
                   uint32_t* n_levels_out)
{
    if (!dims || ndims < 3 || !n_levels_out)
        return -1;
    for (uint32_t i = 0; i < ndims; ++i)
        if (dims[i].chunk_size_px == 0)
            return -1;

    const oracle_dim* x = &dims[ndims - 1];
    const oracle_dim* y = &dims[ndims - 2];
    const oracle_dim* z = &dims[ndims - 3];

    /* :507-520, isotropic assumption -> min over x and y */
    const uint32_t nx = levels_along(x);
    const uint32_t ny = levels_along(y);
    uint32_t n_levels = nx < ny ? nx : ny;

    /* :527-538, a spatial 3rd-from-last dimension may add levels */
    if (z->type == 0 /* Space */) {
        const uint32_t nz = levels_along(z);
        if (nz > n_levels)
            n_levels = nz;
    }

    /* :540-542 */
    if (max_levels > 0 && max_levels < n_levels)
        n_levels = max_levels;

    *n_levels_out = n_levels + 1;
    if (!out)
        return 0;
    if (out_cap_levels < n_levels + 1)
        return -2;

    memcpy(out, dims, ndims * sizeof(oracle_dim));
    for (uint32_t level = 1; level <= n_levels; ++level) {
        const oracle_dim* prev = out + (size_t)(level - 1) * ndims;
        oracle_dim* cur = out + (size_t)level * ndims;

        /* :551-554 non-spatial leading dims copied */
        for (uint32_t i = 0; i + 3 < ndims; ++i)
            cur[i] = prev[i];

        /* :556-563 */
        const oracle_dim* pz = &prev[ndims - 3];
        if (pz->type == 0 && pz->array_size_px > pz->chunk_size_px)
            cur[ndims - 3] = downsample_dimension(*pz);
        else
            cur[ndims - 3] = *pz;

        /* :565-577 */
        const oracle_dim* py = &prev[ndims - 2];
        const oracle_dim* px = &prev[ndims - 1];
        const uint32_t min_size =
          py->array_size_px < px->array_size_px ? py->array_size_px
                                                : px->array_size_px;
        const uint32_t max_chunk =
          py->chunk_size_px > px->chunk_size_px ? py->chunk_size_px
                                                : px->chunk_size_px;
        if (min_size > max_chunk) {
            cur[ndims - 2] = downsample_dimension(*py);
            cur[ndims - 1] = downsample_dimension(*px);
        } else {
            cur[ndims - 2] = *py;
            cur[ndims - 1] = *px;
        }
    }
    return 0;
}

/* ---- stateful downsampler (downsampler.cpp:306-414, 599-605) ---------- */

struct oracle_ds
{
    int dtype, method;
    uint32_t n_levels;
    size_t bpp;
    uint32_t* width;
    uint32_t* height;
    uint32_t* planes;
    uint32_t* count;      /* level_frame_count_ */
    uint8_t** cached;     /* downsampled_frames_ (NULL = absent) */
    size_t* cached_bytes;
    uint8_t** partial;    /* partial_scaled_frames_ (NULL = absent) */
};

oracle_ds*
oracle_ds_create(const uint32_t* widths,
                 const uint32_t* heights,
                 const uint32_t* planes,
                 uint32_t n_levels,
                 int dtype,
                 int method)
{
    if (!widths || !heights || !planes || n_levels == 0)
        return NULL;
    if (oracle_bytes_of_type(dtype) == 0 || method < 0 || method >= M_COUNT)
        return NULL;
    oracle_ds* ds = (oracle_ds*)calloc(1, sizeof(oracle_ds));
    ds->dtype = dtype;
    ds->method = method;
    ds->n_levels = n_levels;
    ds->bpp = oracle_bytes_of_type(dtype);
    ds->width = (uint32_t*)calloc(n_levels, sizeof(uint32_t));
    ds->height = (uint32_t*)calloc(n_levels, sizeof(uint32_t));
    ds->planes = (uint32_t*)calloc(n_levels, sizeof(uint32_t));
    ds->count = (uint32_t*)calloc(n_levels, sizeof(uint32_t));
    ds->cached = (uint8_t**)calloc(n_levels, sizeof(uint8_t*));
    ds->cached_bytes = (size_t*)calloc(n_levels, sizeof(size_t));
    ds->partial = (uint8_t**)calloc(n_levels, sizeof(uint8_t*));
    memcpy(ds->width, widths, n_levels * sizeof(uint32_t));
    memcpy(ds->height, heights, n_levels * sizeof(uint32_t));
    memcpy(ds->planes, planes, n_levels * sizeof(uint32_t));
    return ds;
}

void
oracle_ds_destroy(oracle_ds* ds)
{
    if (!ds)
        return;
    for (uint32_t i = 0; i < ds->n_levels; ++i) {
        free(ds->cached[i]);
        free(ds->partial[i]);
    }
    free(ds->width);
    free(ds->height);
    free(ds->planes);
    free(ds->count);
    free(ds->cached);
    free(ds->cached_bytes);
    free(ds->partial);
    free(ds);
}

/* emplace_downsampled_frame_, downsampler.cpp:599-605: std::unordered_map::
 * emplace never overwrites an untaken frame, but the count always moves. */
static void
emplace_frame(oracle_ds* ds, uint32_t level, uint8_t* frame, size_t bytes)
{
    if (!ds->cached[level]) {
        ds->cached[level] = (uint8_t*)malloc(bytes ? bytes : 1);
        memcpy(ds->cached[level], frame, bytes);
        ds->cached_bytes[level] = bytes;
    }
    ++ds->count[level];
}

int
oracle_ds_add_frame(oracle_ds* ds, const void* frame, size_t nbytes)
{
    size_t fw = ds->width[0], fh = ds->height[0];
    if (nbytes != fw * fh * ds->bpp)
        return -1;
    ++ds->count[0]; /* :311 */

    size_t cur_bytes = nbytes;
    uint8_t* current = (uint8_t*)malloc(cur_bytes ? cur_bytes : 1); /* :314 */
    memcpy(current, frame, nbytes);

    for (uint32_t level = 1; level < ds->n_levels; ++level) {
        const size_t prev_w = ds->width[level - 1];
        const size_t prev_h = ds->height[level - 1];
        const uint32_t prev_planes = ds->planes[level - 1];
        if (prev_w != fw || prev_h != fh) { /* :323-331 */
            free(current);
            return -1;
        }
        const size_t next_w = ds->width[level];
        const size_t next_h = ds->height[level];
        const uint32_t next_planes = ds->planes[level];

        uint8_t* next;
        size_t next_bytes;
        if (next_w < prev_w || next_h < prev_h) { /* :339-343 */
            const size_t ow = (fw + fw % 2) / 2, oh = (fh + fh % 2) / 2;
            next_bytes = ow * oh * ds->bpp;
            next = (uint8_t*)calloc(next_bytes ? next_bytes : 1, 1);
            oracle_scale_image(ds->dtype, ds->method, current, fw, fh, next);
            fw = ow;
            fh = oh;
        } else { /* :344-346 */
            next_bytes = cur_bytes;
            next = (uint8_t*)malloc(next_bytes ? next_bytes : 1);
            memcpy(next, current, next_bytes);
        }
        if (next_w != fw || next_h != fh) { /* :348-356 */
            free(next);
            free(current);
            return -1;
        }

        /* :358-364 */
        int average_this_frame = next_planes < prev_planes;
        if (prev_planes % 2 != 0 && ds->count[level - 1] % prev_planes == 0)
            average_this_frame = 0;

        if (average_this_frame) { /* :368-390 */
            if (ds->partial[level]) {
                /* swap: dst = stored (earlier) plane, src = current */
                uint8_t* earlier = ds->partial[level];
                oracle_average_two_frames(ds->dtype, ds->method, earlier, next,
                                          next_bytes / ds->bpp);
                emplace_frame(ds, level, earlier, next_bytes);
                ds->partial[level] = NULL;
                free(next);
                free(current);
                current = earlier;
                cur_bytes = next_bytes;
            } else {
                ds->partial[level] = next;
                break;
            }
        } else { /* :391-399 */
            emplace_frame(ds, level, next, next_bytes);
            free(current);
            current = next;
            cur_bytes = next_bytes;
        }
    }
    free(current);
    return 0;
}

int
oracle_ds_take_frame(oracle_ds* ds,
                     uint32_t level,
                     void* dst,
                     size_t cap,
                     size_t* nbytes)
{
    /* downsampler.cpp:403-414 */
    if (level >= ds->n_levels)
        return -1;
    if (!ds->cached[level])
        return 0;
    if (cap < ds->cached_bytes[level])
        return -1;
    memcpy(dst, ds->cached[level], ds->cached_bytes[level]);
    if (nbytes)
        *nbytes = ds->cached_bytes[level];
    free(ds->cached[level]);
    ds->cached[level] = NULL;
    return 1;
}

uint32_t
oracle_ds_level_count(const oracle_ds* ds, uint32_t level)
{
    return level < ds->n_levels ? ds->count[level] : 0;
}

/* ---- chunk tiling (array.cpp:507-622, chunk.cpp:17-58) ----------------- */

int
oracle_tile_frame(int dtype,
                  const void* src,
                  uint32_t width,
                  uint32_t height,
                  uint32_t tile_rows,
                  uint32_t tile_cols,
                  void* dst,
                  uint8_t* nonzero)
{
    const size_t bpp = oracle_bytes_of_type(dtype);
    if (!bpp || !src || !dst || tile_rows == 0 || tile_cols == 0)
        return -1;
    const uint32_t n_tiles_x = (width + tile_cols - 1) / tile_cols;
    const uint32_t n_tiles_y = (height + tile_rows - 1) / tile_rows;
    const size_t tile_bytes = (size_t)tile_rows * tile_cols * bpp;
    const size_t src_row_stride = (size_t)width * bpp;
    const size_t dst_row_stride = (size_t)tile_cols * bpp; /* bytes_per_tile_row */
    memset(dst, 0, tile_bytes * n_tiles_x * n_tiles_y);
    for (uint32_t t = 0; t < n_tiles_x * n_tiles_y; ++t) {
        const uint32_t ty = t / n_tiles_x, tx = t % n_tiles_x;
        const uint32_t row0 = ty * tile_rows;
        uint8_t any = 0;
        if (row0 < height) {
            const uint32_t n_rows =
              tile_rows < height - row0 ? tile_rows : height - row0;
            const uint32_t col0 = tx * tile_cols;
            const uint32_t end = col0 + tile_cols < width ? col0 + tile_cols : width;
            const size_t copy = (size_t)(end - col0) * bpp;
            const uint8_t* s = (const uint8_t*)src +
                               ((size_t)row0 * width + col0) * bpp;
            uint8_t* d = (uint8_t*)dst + t * tile_bytes;
            for (uint32_t r = 0; r < n_rows; ++r) {
                const uint8_t* sr = s + r * src_row_stride;
                memcpy(d + r * dst_row_stride, sr, copy);
                for (size_t b = 0; !any && b < copy; ++b)
                    any = sr[b] != 0;
            }
        }
        if (nonzero)
            nonzero[t] = any;
    }
    return 0;
}

/*
 * transpose_frame (array.cpp:488-504): dst[col][row] = src[row][col], one
 * bytes_per_pixel memcpy per pixel, output src_cols x src_rows.
 */
int
oracle_transpose_frame(int dtype,
                       const void* src,
                       uint32_t src_rows,
                       uint32_t src_cols,
                       void* dst)
{
    const size_t bpp = oracle_bytes_of_type(dtype);
    if (!bpp || !src || !dst)
        return -1;
    for (uint32_t row = 0; row < src_rows; ++row) {
        for (uint32_t col = 0; col < src_cols; ++col) {
            const size_t so = ((size_t)row * src_cols + col) * bpp;
            const size_t d_o = ((size_t)col * src_rows + row) * bpp;
            memcpy((uint8_t*)dst + d_o, (const uint8_t*)src + so, bpp);
        }
    }
    return 0;
}

/* ---- chunk addressing (array.dimensions.cpp:232-314) -------------------- */

/*
 * ArrayDimensions::chunk_lattice_index (array.dimensions.cpp:232-262): the
 * chunk index of frame `frame_id` along non-spatial dim `dim_index`.  Dim 0
 * (the append dimension) divides by its chunk size times the array sizes of
 * dims 1..ndims-3; the others take the frame id modulo the array sizes from
 * dim_index on, divided by dim_index's chunk size times the faster sizes.
 * Returns UINT32_MAX for a dim_index the reference's EXPECT rejects.
 */
uint32_t
oracle_chunk_lattice_index(const oracle_dim* dims,
                           uint32_t ndims,
                           uint64_t frame_id,
                           uint32_t dim_index)
{
    if (!dims || ndims < 3 || dim_index >= ndims - 2)
        return UINT32_MAX;
    if (dim_index == 0) {
        uint64_t divisor = dims[0].chunk_size_px;
        for (uint32_t i = 1; i < ndims - 2; ++i)
            divisor *= dims[i].array_size_px;
        return divisor ? (uint32_t)(frame_id / divisor) : UINT32_MAX;
    }
    uint64_t mod_divisor = 1, div_divisor = 1;
    for (uint32_t i = dim_index; i < ndims - 2; ++i) {
        mod_divisor *= dims[i].array_size_px;
        div_divisor *=
          i == dim_index ? dims[i].chunk_size_px : dims[i].array_size_px;
    }
    if (!mod_divisor || !div_divisor)
        return UINT32_MAX;
    return (uint32_t)((frame_id % mod_divisor) / div_divisor);
}

/*
 * ArrayDimensions::tile_group_offset (array.dimensions.cpp:264-282): the
 * index, in chunks, of the first chunk of the frame's tile group inside its
 * chunk layer — lattice index x chunk-count stride, over dims ndims-3 .. 1.
 */
uint64_t
oracle_tile_group_offset(const oracle_dim* dims, uint32_t ndims, uint64_t frame_id)
{
    if (!dims || ndims < 3)
        return UINT64_MAX;
    uint64_t strides[64];
    if (ndims > 64)
        return UINT64_MAX;
    strides[ndims - 1] = 1;
    for (uint32_t i = ndims - 1; i > 0; --i) {
        const uint64_t a = dims[i].array_size_px, c = dims[i].chunk_size_px;
        if (!c)
            return UINT64_MAX;
        strides[i - 1] = strides[i] * ((a + c - 1) / c);
    }
    uint64_t offset = 0;
    for (uint32_t i = ndims - 3; i > 0; --i)
        offset += (uint64_t)oracle_chunk_lattice_index(dims, ndims, frame_id, i) *
                  strides[i];
    return offset;
}

/*
 * ArrayDimensions::chunk_internal_offset (array.dimensions.cpp:284-314): the
 * byte offset of the frame's tile inside its chunk — its index within the
 * chunk along every non-spatial dim, in chunk strides, times one tile's
 * bytes (bytes_per_px x Y chunk x X chunk).
 */
uint64_t
oracle_chunk_internal_offset(const oracle_dim* dims,
                             uint32_t ndims,
                             uint32_t bytes_per_px,
                             uint64_t frame_id)
{
    if (!dims || ndims < 3 || ndims > 64)
        return UINT64_MAX;
    const uint64_t tile_size = (uint64_t)bytes_per_px *
                               dims[ndims - 1].chunk_size_px *
                               dims[ndims - 2].chunk_size_px;
    uint64_t array_strides[64], chunk_strides[64];
    for (uint32_t i = 0; i < ndims - 2; ++i)
        array_strides[i] = chunk_strides[i] = 1;
    uint64_t offset = 0;
    for (int i = (int)ndims - 3; i > 0; --i) {
        const uint64_t a = dims[i].array_size_px, c = dims[i].chunk_size_px;
        if (!a || !c)
            return UINT64_MAX;
        const uint64_t internal_idx = (frame_id / array_strides[i]) % a % c;
        array_strides[i - 1] = array_strides[i] * a;
        chunk_strides[i - 1] = chunk_strides[i] * c;
        offset += internal_idx * chunk_strides[i];
    }
    if (!dims[0].chunk_size_px)
        return UINT64_MAX;
    offset += (frame_id / array_strides[0]) % dims[0].chunk_size_px * chunk_strides[0];
    return offset * tile_size;
}
