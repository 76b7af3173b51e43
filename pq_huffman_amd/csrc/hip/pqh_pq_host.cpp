// pqh_pq_host.cpp -- pq.h host-pointer entry points (pq_encode, pq_compute_error) staged
// through device memory on a private pqh context.  No CPU fallback: without a GPU they
// return PQH_ERR_NO_DEVICE.
#include <cstdint>

#include "pq.h"
#include "pqh_internal.h"

namespace {
struct Ctx {
    pqh_ctx_t* c = nullptr;
    ~Ctx() { pqh_ctx_destroy(c); }
};
}  // namespace

extern "C" int pq_encode(const centroids_codebook_t* cb, const float* x, long long n, int d,
                         void* codes) {
    if (!cb || !x || !codes || n < 0 || d != cb->num_parts * cb->num_dimensions) return PQH_ERR_ARG;
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
    if (!rc) rc = pqh_pq_assign(ctx, pq, dx, n, d, dc, nullptr, 0);
    if (!rc) rc = pqh_ctx_sync(ctx);
    if (!rc && hipMemcpy(codes, dc, (size_t)n * cb->num_parts * esz, hipMemcpyDeviceToHost) != hipSuccess)
        rc = PQH_ERR_HIP;
    pqh_pq_destroy(pq);
    (void)hipFree(dx);
    (void)hipFree(dc);
    return rc;
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
