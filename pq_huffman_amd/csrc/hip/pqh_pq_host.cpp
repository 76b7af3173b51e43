// pqh_pq_host.cpp -- pq.h host-pointer entry points (pq_encode, pq_compute_error) staged
// through device memory on a private pqh context.  No CPU fallback: without a GPU they
// return PQH_ERR_NO_DEVICE.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "pq.h"
#include "pqh_internal.h"

namespace {
struct Ctx {
    pqh_ctx_t* c = nullptr;
    ~Ctx() { pqh_ctx_destroy(c); }
};
}  // namespace

// The streaming encoder behind pq_encode / pq_encode_rows: rows are taken chunk_rows at a
// time through two pinned host buffers, so device memory stays at two chunks whatever n is
// (the reference, src/pq_encoder.c:43,58-80, reads its input 128K rows at a time).  Chunk
// i's rows are produced by the caller's reader (a file read, a copy) while chunk i - 1 is
// copied in and assigned: H2D and D2H run on a copy stream, the assignment on the context's
// stream, ordered by events.
namespace {
struct Stream {
    hipStream_t copy = nullptr;
    float* hin[2] = {nullptr, nullptr};
    unsigned char* hout[2] = {nullptr, nullptr};
    float* dx[2] = {nullptr, nullptr};
    unsigned char* dc[2] = {nullptr, nullptr};
    hipEvent_t h2d[2] = {nullptr, nullptr}, asg[2] = {nullptr, nullptr}, d2h[2] = {nullptr, nullptr};
    ~Stream() {
        for (int b = 0; b < 2; ++b) {
            if (hin[b]) (void)hipHostFree(hin[b]);
            if (hout[b]) (void)hipHostFree(hout[b]);
            if (dx[b]) (void)hipFree(dx[b]);
            if (dc[b]) (void)hipFree(dc[b]);
            for (hipEvent_t e : {h2d[b], asg[b], d2h[b]})
                if (e) (void)hipEventDestroy(e);
        }
        if (copy) (void)hipStreamDestroy(copy);
    }
};

long long default_chunk_rows() {
    const char* e = std::getenv("PQH_ENCODE_CHUNK");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? v : (1ll << 18);   // 256K rows: 128 MB of 128-d fp32 per buffer
}

struct CopyReader {
    const float* x;
    int d;
};
int copy_rows(void* user, long long row0, long long rows, float* dst) {
    const CopyReader* r = static_cast<const CopyReader*>(user);
    std::memcpy(dst, r->x + row0 * r->d, (size_t)rows * r->d * sizeof(float));
    return 0;
}
}  // namespace

extern "C" int pq_encode_rows(const centroids_codebook_t* cb, int d, long long n,
                              pq_rows_fn read, void* user, void* codes, long long chunk_rows) {
    if (!cb || !read || !codes || n < 0 || d != cb->num_parts * cb->num_dimensions) return PQH_ERR_ARG;
    if (n == 0) return PQH_OK;
    if (chunk_rows <= 0) chunk_rows = default_chunk_rows();
    chunk_rows = std::min(chunk_rows, n);
    Ctx g;
    int rc = pqh_ctx_create(&g.c, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.c;
    pqh_pq_t* pq = nullptr;
    rc = pqh_pq_create(ctx, cb->centroids_pool, cb->num_parts, cb->num_clusters, cb->num_dimensions, &pq);
    if (rc) return rc;
    struct PqGuard {
        pqh_pq_t* p;
        ~PqGuard() { pqh_pq_destroy(p); }
    } pg{pq};
    const size_t esz = cb->num_clusters <= 256 ? 1 : 2;
    const size_t xbytes = (size_t)chunk_rows * d * sizeof(float), cbytes = (size_t)chunk_rows * cb->num_parts * esz;
    Stream st;
    if (hipStreamCreateWithFlags(&st.copy, hipStreamNonBlocking) != hipSuccess) return PQH_ERR_HIP;
    for (int b = 0; b < 2; ++b) {
        if (hipHostMalloc(reinterpret_cast<void**>(&st.hin[b]), xbytes, 0) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&st.hout[b]), cbytes, 0) != hipSuccess ||
            hipMalloc(&st.dx[b], xbytes + 16) != hipSuccess || hipMalloc(&st.dc[b], cbytes + 16) != hipSuccess)
            return PQH_ERR_NOMEM;
        for (hipEvent_t* e : {&st.h2d[b], &st.asg[b], &st.d2h[b]})
            if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return PQH_ERR_HIP;
    }
    const long long chunks = (n + chunk_rows - 1) / chunk_rows;
    unsigned char* out = static_cast<unsigned char*>(codes);
    const size_t row_code = (size_t)cb->num_parts * esz;
    auto finish = [&](long long i) -> int {   // chunk i's codes: wait for its D2H, hand out
        const int b = (int)(i & 1);
        if (hipEventSynchronize(st.d2h[b]) != hipSuccess) return PQH_ERR_HIP;
        const long long r0 = i * chunk_rows, rows = std::min(chunk_rows, n - r0);
        std::memcpy(out + (size_t)r0 * row_code, st.hout[b], (size_t)rows * row_code);
        return PQH_OK;
    };
    for (long long i = 0; i < chunks && !rc; ++i) {
        const int b = (int)(i & 1);
        const long long r0 = i * chunk_rows, rows = std::min(chunk_rows, n - r0);
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
        if ((rc = pqh_pq_assign(ctx, pq, st.dx[b], rows, d, st.dc[b], nullptr, 0))) break;
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

extern "C" int pq_compute_error(const centroids_codebook_t* cb, const float* x, long long n, int d,
                                const void* codes, double* error_out) {
    if (!cb || !x || !codes || !error_out || n <= 0 || d != cb->num_parts * cb->num_dimensions)
        return PQH_ERR_ARG;
    Ctx g;
    int rc = pqh_ctx_create(&g.c, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.c;
    pqh_pq_t* pq = nullptr;
    rc = pqh_pq_create(ctx, cb->centroids_pool, cb->num_parts, cb->num_clusters, cb->num_dimensions, &pq);
    if (rc) return rc;
    const size_t esz = cb->num_clusters <= 256 ? 1 : 2;
    float* dx = nullptr;
    void* dc = nullptr;
    if (hipMalloc(&dx, (size_t)n * d * 4 + 16) != hipSuccess ||
        hipMalloc(&dc, (size_t)n * cb->num_parts * esz + 16) != hipSuccess) {
        pqh_pq_destroy(pq);
        if (dx) (void)hipFree(dx);
        return PQH_ERR_NOMEM;
    }
    rc = hipMemcpy(dx, x, (size_t)n * d * 4, hipMemcpyHostToDevice) == hipSuccess ? PQH_OK : PQH_ERR_HIP;
    if (!rc && hipMemcpy(dc, codes, (size_t)n * cb->num_parts * esz, hipMemcpyHostToDevice) != hipSuccess)
        rc = PQH_ERR_HIP;
    if (!rc) rc = pqh_pq_error(ctx, pq, dx, n, d, dc, error_out);
    pqh_pq_destroy(pq);
    (void)hipFree(dx);
    (void)hipFree(dc);
    return rc;
}

// k-means training of the whole codebook on the GPU (pqh_kmeans_train); the codebook holds
// the initial centroids on entry and the trained ones on return
extern "C" int pq_train(centroids_codebook_t* cb, const float* x, long long n, int d, int iters) {
    if (!cb || !x || n < 0 || iters < 0 || d != cb->num_parts * cb->num_dimensions) return PQH_ERR_ARG;
    Ctx g;
    int rc = pqh_ctx_create(&g.c, 0);
    if (rc) return rc;
    float* dx = nullptr;
    if (hipMalloc(&dx, (size_t)n * d * 4 + 16) != hipSuccess) return PQH_ERR_NOMEM;
    rc = hipMemcpy(dx, x, (size_t)n * d * 4, hipMemcpyHostToDevice) == hipSuccess ? PQH_OK : PQH_ERR_HIP;
    if (!rc)
        rc = pqh_kmeans_train(g.c, dx, n, d, cb->num_parts, cb->num_clusters, cb->num_dimensions,
                              iters, cb->centroids_pool);
    (void)hipFree(dx);
    return rc;
}
