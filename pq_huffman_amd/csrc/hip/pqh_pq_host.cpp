// pqh_pq_host.cpp -- pq.h host-pointer entry points (pq_encode[_rows], pq_train[_rows],
// pq_compute_error[_rows]) staged through device memory on a private pqh context.  Every
// pass streams the rows a chunk at a time, so device memory stays at two chunks whatever n
// is (the reference reads its input in 128K-row batches, src/pq_encoder.c:43,58-80,89-113).
// No CPU fallback: without a GPU they return PQH_ERR_NO_DEVICE.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pq.h"
#include "pqh_internal.h"

namespace {
struct Ctx {
    pqh_ctx_t* c = nullptr;
    ~Ctx() { pqh_ctx_destroy(c); }
};

struct PqGuard {
    pqh_pq_t* p = nullptr;
    ~PqGuard() { pqh_pq_destroy(p); }
};

// Rows per chunk: PQH_ENCODE_CHUNK, else 2^18 rows capped at 128 MB of fp32 per buffer (at
// d = 960 that is 34,952 rows, not 2^18 rows = 1 GB), rounded down to a multiple of 256 so
// the error pass's 256-row blocks line up with the one-shot pass's.
long long chunk_rows_for(int d, long long requested, long long n) {
    long long c = requested;
    if (c <= 0) {
        const char* e = std::getenv("PQH_ENCODE_CHUNK");
        c = e ? std::atoll(e) : 0;
    }
    if (c <= 0) c = std::min<long long>(1ll << 18, (128ll << 20) / (4ll * std::max(d, 1)));
    c = std::max<long long>(256, (c / 256) * 256);
    return std::max<long long>(1, std::min(c, n));
}

// Two pinned host buffers and two device buffers of `chunk` rows (+ codes), events to
// order them.  alloc() halves the chunk (in multiples of 256 rows) on an allocation failure
// before giving up with PQH_ERR_NOMEM.
struct Pump {
    hipStream_t copy = nullptr;
    float* hin[2] = {nullptr, nullptr};
    unsigned char* hout[2] = {nullptr, nullptr};
    float* dx[2] = {nullptr, nullptr};
    unsigned char* dc[2] = {nullptr, nullptr};
    hipEvent_t h2d[2] = {nullptr, nullptr}, asg[2] = {nullptr, nullptr}, d2h[2] = {nullptr, nullptr};
    long long chunk = 0;
    void release() {
        for (int b = 0; b < 2; ++b) {
            if (hin[b]) (void)hipHostFree(hin[b]);
            if (hout[b]) (void)hipHostFree(hout[b]);
            if (dx[b]) (void)hipFree(dx[b]);
            if (dc[b]) (void)hipFree(dc[b]);
            hin[b] = nullptr;
            hout[b] = nullptr;
            dx[b] = nullptr;
            dc[b] = nullptr;
        }
    }
    ~Pump() {
        release();
        for (int b = 0; b < 2; ++b)
            for (hipEvent_t e : {h2d[b], asg[b], d2h[b]})
                if (e) (void)hipEventDestroy(e);
        if (copy) (void)hipStreamDestroy(copy);
    }
    // code_bytes: per row (0: no code buffers); host_codes: pinned host code buffers too
    int alloc(long long rows, int d, size_t code_bytes, bool host_codes) {
        if (!copy && hipStreamCreateWithFlags(&copy, hipStreamNonBlocking) != hipSuccess)
            return PQH_ERR_HIP;
        for (int b = 0; b < 2; ++b)
            for (hipEvent_t* e : {&h2d[b], &asg[b], &d2h[b]})
                if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess)
                    return PQH_ERR_HIP;
        // (never below 256 rows, or below the whole input when it is shorter: the error
        // pass's 256-row block partials must line up with the one-shot pass's -- pq.h)
        const long long floor_rows = std::min<long long>(rows, 256);
        for (chunk = rows; chunk >= floor_rows; chunk = ((chunk / 2 + 255) / 256) * 256) {
            const size_t xb = (size_t)chunk * d * sizeof(float), cb = (size_t)chunk * code_bytes;
            bool ok = true;
            for (int b = 0; b < 2 && ok; ++b) {
                ok = hipHostMalloc(reinterpret_cast<void**>(&hin[b]), xb, 0) == hipSuccess &&
                     hipMalloc(&dx[b], xb + 16) == hipSuccess;
                if (ok && code_bytes) ok = hipMalloc(&dc[b], cb + 16) == hipSuccess;
                if (ok && code_bytes && host_codes)
                    ok = hipHostMalloc(reinterpret_cast<void**>(&hout[b]), cb, 0) == hipSuccess;
            }
            if (ok) return PQH_OK;
            release();
            (void)hipGetLastError();   // (clear the failed allocation's sticky error)
            if (chunk <= floor_rows) break;
        }
        return PQH_ERR_NOMEM;
    }
};

struct CopyReader {
    const float* x;
    int d;
};
int copy_rows(void* user, long long row0, long long rows, float* dst) {
    const CopyReader* r = static_cast<const CopyReader*>(user);
    std::memcpy(dst, r->x + row0 * r->d, (size_t)rows * r->d * sizeof(float));
    return 0;
}

// One pass over the rows on ctx's stream: chunk i is read into pinned buffer i & 1 (while the
// device works on chunk i - 1), copied in, and handed to work(i, d_x, row0, rows, b), which
// enqueues its kernels on ctx->stream.  Returns after the last chunk's work is enqueued.
template <class F>
int pass(pqh_ctx* ctx, Pump& p, int d, long long n, pq_rows_fn read, void* user, F&& work) {
    const long long chunks = (n + p.chunk - 1) / p.chunk;
    for (long long i = 0; i < chunks; ++i) {
        const int b = (int)(i & 1);
        const long long r0 = i * p.chunk, rows = std::min(p.chunk, n - r0);
        if (i >= 2 && hipEventSynchronize(p.asg[b]) != hipSuccess) return PQH_ERR_HIP;
        if (read(user, r0, rows, p.hin[b]))
            return pqh_set_error(ctx, PQH_ERR_ARG, "the row reader failed at row %lld", r0);
        if (hipMemcpyAsync(p.dx[b], p.hin[b], (size_t)rows * d * sizeof(float),
                           hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
            return PQH_ERR_HIP;
        const int rc = work(i, p.dx[b], r0, rows, b);
        if (rc) return rc;
        if (hipEventRecord(p.asg[b], ctx->stream) != hipSuccess) return PQH_ERR_HIP;
    }
    return hipStreamSynchronize(ctx->stream) == hipSuccess ? PQH_OK : PQH_ERR_HIP;
}
}  // namespace

// The streaming encoder behind pq_encode / pq_encode_rows.  Chunk i's rows are produced by
// the caller's reader (a file read, a copy) while chunk i - 1 is copied in and assigned:
// H2D and D2H run on a copy stream, the assignment on the context's stream, ordered by events.
extern "C" int pq_encode_rows(const centroids_codebook_t* cb, int d, long long n,
                              pq_rows_fn read, void* user, void* codes, long long chunk_rows) {
    if (!cb || !read || !codes || n < 0 || d != cb->num_parts * cb->num_dimensions) return PQH_ERR_ARG;
    if (n == 0) return PQH_OK;
    Ctx g;
    int rc = pqh_ctx_create(&g.c, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.c;
    PqGuard pg;
    rc = pqh_pq_create(ctx, cb->centroids_pool, cb->num_parts, cb->num_clusters, cb->num_dimensions, &pg.p);
    if (rc) return rc;
    const size_t esz = cb->num_clusters <= 256 ? 1 : 2;
    const size_t row_code = (size_t)cb->num_parts * esz;
    Pump st;
    if ((rc = st.alloc(chunk_rows_for(d, chunk_rows, n), d, row_code, true))) return rc;
    const long long chunk = st.chunk;
    const long long chunks = (n + chunk - 1) / chunk;
    unsigned char* out = static_cast<unsigned char*>(codes);
    auto finish = [&](long long i) -> int {   // chunk i's codes: wait for its D2H, hand out
        const int b = (int)(i & 1);
        if (hipEventSynchronize(st.d2h[b]) != hipSuccess) return PQH_ERR_HIP;
        const long long r0 = i * chunk, rows = std::min(chunk, n - r0);
        std::memcpy(out + (size_t)r0 * row_code, st.hout[b], (size_t)rows * row_code);
        return PQH_OK;
    };
    for (long long i = 0; i < chunks && !rc; ++i) {
        const int b = (int)(i & 1);
        const long long r0 = i * chunk, rows = std::min(chunk, n - r0);
        if (i >= 2 && (rc = finish(i - 2))) break;   // buffer set b is free again
        if (read(user, r0, rows, st.hin[b])) {
            rc = pqh_set_error(ctx, PQH_ERR_ARG, "pq_encode_rows: the row reader failed at row %lld", r0);
            break;
        }
        if (hipMemcpyAsync(st.dx[b], st.hin[b], (size_t)rows * d * sizeof(float),
                           hipMemcpyHostToDevice, st.copy) != hipSuccess ||
            hipEventRecord(st.h2d[b], st.copy) != hipSuccess ||
            hipStreamWaitEvent(ctx->stream, st.h2d[b], 0) != hipSuccess) {
            rc = PQH_ERR_HIP;
            break;
        }
        if ((rc = pqh_pq_assign(ctx, pg.p, st.dx[b], rows, d, st.dc[b], nullptr, 0))) break;
        if (hipEventRecord(st.asg[b], ctx->stream) != hipSuccess ||
            hipStreamWaitEvent(st.copy, st.asg[b], 0) != hipSuccess ||
            hipMemcpyAsync(st.hout[b], st.dc[b], (size_t)rows * row_code, hipMemcpyDeviceToHost,
                           st.copy) != hipSuccess ||
            hipEventRecord(st.d2h[b], st.copy) != hipSuccess)
            rc = PQH_ERR_HIP;
    }
    for (long long i = std::max(0ll, chunks - 2); i < chunks && !rc; ++i) rc = finish(i);
    (void)hipStreamSynchronize(st.copy);
    (void)hipStreamSynchronize(ctx->stream);
    return rc;
}

extern "C" int pq_encode(const centroids_codebook_t* cb, const float* x, long long n, int d,
                         void* codes) {
    if (!cb || !x || !codes || n < 0 || d != cb->num_parts * cb->num_dimensions) return PQH_ERR_ARG;
    CopyReader r{x, d};
    return pq_encode_rows(cb, d, n, copy_rows, &r, codes, 0);
}

// compute_error (src/pq_encoder.c:82-119) streamed: each chunk's codes go in beside its rows,
// pqh_pq_error_accum adds the chunk's 256-row block partials in row order -- the one-shot
// pqh_pq_error's sum bit for bit, since chunks hold whole blocks.
extern "C" int pq_compute_error_rows(const centroids_codebook_t* cb, int d, long long n,
                                     pq_rows_fn read, void* user, const void* codes,
                                     long long chunk_rows, double* error_out) {
    if (!cb || !read || !codes || !error_out || n <= 0 || d != cb->num_parts * cb->num_dimensions)
        return PQH_ERR_ARG;
    Ctx g;
    int rc = pqh_ctx_create(&g.c, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.c;
    PqGuard pg;
    rc = pqh_pq_create(ctx, cb->centroids_pool, cb->num_parts, cb->num_clusters, cb->num_dimensions, &pg.p);
    if (rc) return rc;
    const size_t row_code = (size_t)cb->num_parts * (cb->num_clusters <= 256 ? 1 : 2);
    Pump p;
    if ((rc = p.alloc(chunk_rows_for(d, chunk_rows, n), d, row_code, false))) return rc;
    const unsigned char* hc = static_cast<const unsigned char*>(codes);
    double sum = 0.0;
    rc = pass(ctx, p, d, n, read, user, [&](long long, float* dx, long long r0, long long rows, int b) {
        if (hipMemcpyAsync(p.dc[b], hc + (size_t)r0 * row_code, (size_t)rows * row_code,
                           hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
            return (int)PQH_ERR_HIP;
        // (synchronises: the partials are summed on the host in row order)
        return pqh_pq_error_accum(ctx, pg.p, dx, rows, d, p.dc[b], &sum);
    });
    if (rc) return rc;
    *error_out = sum / (double)n;
    return PQH_OK;
}

extern "C" int pq_compute_error(const centroids_codebook_t* cb, const float* x, long long n, int d,
                                const void* codes, double* error_out) {
    if (!cb || !x || !codes || !error_out || n <= 0 || d != cb->num_parts * cb->num_dimensions)
        return PQH_ERR_ARG;
    CopyReader r{x, d};
    return pq_compute_error_rows(cb, d, n, copy_rows, &r, codes, 0, error_out);
}

// k-means training (pqh_kmeans_train's Lloyd) streamed: one pass for max |x| (the fixed-point
// shift), then per iteration one pass assigning each chunk and adding its fixed-point sums --
// exact integers, so the result equals pqh_kmeans_train on all rows at once, bit for bit.
extern "C" int pq_train_rows(centroids_codebook_t* cb, int d, long long n, pq_rows_fn read,
                             void* user, int iters, long long chunk_rows) {
    if (!cb || !read || n < 0 || iters < 0 || d != cb->num_parts * cb->num_dimensions)
        return PQH_ERR_ARG;
    if (n == 0 || iters == 0) return PQH_OK;
    Ctx g;
    int rc = pqh_ctx_create(&g.c, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.c;
    const int m = cb->num_parts, k = cb->num_clusters, dsub = cb->num_dimensions;
    const long long cells = (long long)m * k;
    const size_t row_code = (size_t)m * (k <= 256 ? 1 : 2);
    Pump p;
    if ((rc = p.alloc(chunk_rows_for(d, chunk_rows, n), d, row_code, false))) return rc;
    struct Dev {
        long long* sums = nullptr;
        unsigned long long* cnt = nullptr;
        float* cent = nullptr;
        unsigned* mx = nullptr;
        ~Dev() {
            (void)hipFree(sums);
            (void)hipFree(cnt);
            (void)hipFree(cent);
            (void)hipFree(mx);
        }
    } dv;
    if (hipMalloc(&dv.sums, (size_t)cells * dsub * 8) != hipSuccess ||
        hipMalloc(&dv.cnt, (size_t)cells * 8) != hipSuccess ||
        hipMalloc(&dv.cent, (size_t)cells * dsub * 4) != hipSuccess || hipMalloc(&dv.mx, 4) != hipSuccess)
        return pqh_set_error(ctx, PQH_ERR_NOMEM, "kmeans buffers");
    PQH_HIP(ctx, hipMemsetAsync(dv.mx, 0, 4, ctx->stream));
    rc = pass(ctx, p, d, n, read, user, [&](long long, float* dx, long long, long long rows, int) {
        return pqh_kmeans_absmax_launch(ctx, dx, rows, d, d, dv.mx);
    });
    if (rc) return rc;
    unsigned hmax = 0;
    PQH_HIP(ctx, hipMemcpy(&hmax, dv.mx, 4, hipMemcpyDeviceToHost));
    float fmax;
    std::memcpy(&fmax, &hmax, 4);
    const int s = pqh_kmeans_fixed_shift(fmax, n);
    for (int it = 0; it < iters; ++it) {
        PqGuard pg;
        if ((rc = pqh_pq_create(ctx, cb->centroids_pool, m, k, dsub, &pg.p))) return rc;
        PQH_HIP(ctx, hipMemsetAsync(dv.sums, 0, (size_t)cells * dsub * 8, ctx->stream));
        PQH_HIP(ctx, hipMemsetAsync(dv.cnt, 0, (size_t)cells * 8, ctx->stream));
        PQH_HIP(ctx, hipMemcpyAsync(dv.cent, cb->centroids_pool, (size_t)cells * dsub * 4,
                                    hipMemcpyHostToDevice, ctx->stream));
        rc = pass(ctx, p, d, n, read, user, [&](long long, float* dx, long long, long long rows, int b) {
            int r = pqh_pq_assign(ctx, pg.p, dx, rows, d, p.dc[b], nullptr, 0);
            if (!r) r = pqh_kmeans_accum_launch(ctx, dx, rows, d, m, k, dsub, p.dc[b], s, dv.sums, dv.cnt);
            return r;
        });
        if (rc) return rc;
        if ((rc = pqh_kmeans_update_launch(ctx, dv.sums, dv.cnt, cells, dsub, s, dv.cent))) return rc;
        PQH_HIP(ctx, hipMemcpyAsync(cb->centroids_pool, dv.cent, (size_t)cells * dsub * 4,
                                    hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return PQH_OK;
}

// k-means training of the whole codebook on the GPU; the codebook holds the initial centroids
// on entry and the trained ones on return
extern "C" int pq_train(centroids_codebook_t* cb, const float* x, long long n, int d, int iters) {
    if (!cb || !x || n < 0 || iters < 0 || d != cb->num_parts * cb->num_dimensions) return PQH_ERR_ARG;
    CopyReader r{x, d};
    return pq_train_rows(cb, d, n, copy_rows, &r, iters, 0);
}
