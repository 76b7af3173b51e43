/*
 * pq.h -- the reference ships this header EMPTY (src/pq.h, 0 bytes; the PQ helpers are
 * `static` in pq_encoder.c:34-255 with "TODO: Move to library part" at :226).  This is
 * the library surface the build defines for it:
 *   - centroids_codebook_t with the layout of pq_encoder.c:34-40 and its init/destroy/
 *     save (pq_encoder.c:227-255) plus load;
 *   - .fvecs reading in ONE pass (the reference re-reads the file once per subspace,
 *     pq_encoder.c:58-80,265-269);
 *   - pq_encode: nearest-centroid assignment, which the reference does inside yael
 *     kmeans() (pq_encoder.c:270-272), run on the GPU by pqh_pq_assign (pqh.h);
 *   - pq_compute_error (pq_encoder.c:82-119) on the GPU.
 * Host-pointer convenience wrappers: they stage through device memory on the default
 * pqh context.  Return 0 on success, a negative pqh_status_t otherwise (never assert).
 */
#ifndef _PQ_H
#define _PQ_H

#include "misc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _centroids_codebook {
    int num_clusters;      /* K */
    int num_dimensions;    /* dsub = D / M */
    int num_parts;         /* M */
    float* centroids_pool; /* [M][K][dsub] */
    float** centroids;     /* per-part pointers into the pool */
} centroids_codebook_t;

void centroids_codebook_init(centroids_codebook_t* codebook, int num_parts, int num_clusters,
                             int num_dimensions);
void centroids_codebook_destroy(centroids_codebook_t* codebook);
/* pq_centroids.fvecsl: u32 M*K, u32 dsub, float[M][K][dsub] (pq_encoder.c:248-255) */
int centroids_codebook_save(const centroids_codebook_t* codebook, const char* filename);
int centroids_codebook_load(centroids_codebook_t* codebook, const char* filename, int num_parts,
                            int num_clusters);

/* .fvecs: per row i32 D + float[D] (pq_encoder.c:46-80).  N = file size / (4 + 4D). */
int fvecs_load_meta(const char* filename, long long* num_vectors, int* num_dimensions);
float* fvecs_load(const char* filename, long long* num_vectors, int* num_dimensions);

/* codes: n x M, uint8 when K <= 256 else uint16 (row-major, pq_indices.bvecsl order).
 * Streams: the rows go to the GPU a chunk at a time (PQH_ENCODE_CHUNK rows, default 2^18
 * capped at 128 MB of rows per buffer, halved on an allocation failure) through two pinned
 * buffers, so device memory is bounded for any n. */
int pq_encode(const centroids_codebook_t* codebook, const float* x, long long n, int d,
              void* codes);
/* pq_encode over rows produced by the caller: read(user, row0, rows, dst) fills rows
 * [row0, row0 + rows) as rows x d floats into dst (a pinned buffer) and returns 0; the
 * reader for chunk i + 1 runs while chunk i is copied and assigned (the pq_encoder CLI reads
 * its .fvecs file this way, as the reference does in 128K-row batches, pq_encoder.c:43,58-80).
 * chunk_rows <= 0: the default. */
typedef int (*pq_rows_fn)(void* user, long long row0, long long rows, float* dst);
int pq_encode_rows(const centroids_codebook_t* codebook, int d, long long n, pq_rows_fn read,
                   void* user, void* codes, long long chunk_rows);
/* Train the codebook in place on the GPU: `iters` deterministic Lloyd iterations
 * (pqh_kmeans_train) from the centroids it holds -- the build's replacement for the
 * training done by yael kmeans at pq_encoder.c:265-274.  Streams like pq_encode. */
int pq_train(centroids_codebook_t* codebook, const float* x, long long n, int d, int iters);
/* pq_train over rows produced by the caller (read as for pq_encode_rows): one pass for the
 * fixed-point scale, then one pass per iteration; device memory stays at two chunks for any
 * n, and the centroids equal pq_train's on the same rows bit for bit (exact fixed-point
 * sums).  The reference holds one N x dsub slice at a time (pq_encoder.c:265-269). */
int pq_train_rows(centroids_codebook_t* codebook, int d, long long n, pq_rows_fn read,
                  void* user, int iters, long long chunk_rows);
/* mean over vectors of the summed squared reconstruction error (double), as
 * compute_error (pq_encoder.c:82-119). */
int pq_compute_error(const centroids_codebook_t* codebook, const float* x, long long n, int d,
                     const void* codes, double* error_out);
/* pq_compute_error over rows produced by the caller, a chunk at a time (the reference reads
 * 128K-row batches, pq_encoder.c:89-113); codes are the n x M host codes.  The result equals
 * pq_compute_error's bit for bit (256-row partial sums added in row order). */
int pq_compute_error_rows(const centroids_codebook_t* codebook, int d, long long n,
                          pq_rows_fn read, void* user, const void* codes, long long chunk_rows,
                          double* error_out);

#ifdef __cplusplus
}
#endif

#endif /* _PQ_H */
