/* pq_encoder -- CLI-compatible replacement for the reference's src/pq_encoder.c
 * (usage pq_encoder.c:121-175; outputs :207-213, :248-255, :290-295).
 *   pq_encoder <input.fvecs> <output template> <m> [--num-threads t] [--compute-error]
 *              [--kmeans-iterations n] [--centroids <pq_centroids.fvecsl>] [--seed s]
 * Assignment and training run on the GPU (libpqh).  Training: deterministic Lloyd
 * iterations on the GPU (pq_train_rows: exact assignment, fixed-point centroid means) from a
 * seeded sample init (yael's time-seeded Berkeley init is not reproducible); --centroids
 * skips training.  Training, encoding and --compute-error all stream the file in chunks
 * (PQH_ENCODE_CHUNK rows), so neither host nor device memory holds the input whole.
 * --num-threads is accepted for compatibility. */
#define _FILE_OFFSET_BITS 64
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "misc.h"
#include "pq.h"
#include "vecs_io.h"

static unsigned long long rng_state = 0x9E3779B97F4A7C15ULL;
static unsigned long long rng_next(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

/* Streaming .fvecs reader for pq_encode_rows: rows [row0, row0 + rows) into dst, the
 * per-row i32 dimension headers dropped (pq_encoder.c:58-80 reads 128K-row batches). */
typedef struct {
    FILE* f;
    int d;
    int32_t* raw;
    long long cap;    /* rows of raw */
    long long next;   /* the row the file position is at */
} fvecs_reader_t;

static int fvecs_rows(void* user, long long row0, long long rows, float* dst) {
    fvecs_reader_t* r = (fvecs_reader_t*)user;
    const long long rb = 4LL * (r->d + 1);
    if (row0 != r->next && fseeko(r->f, (off_t)(row0 * rb), SEEK_SET)) return -1;
    r->next = row0;
    while (rows > 0) {
        const long long want = rows < r->cap ? rows : r->cap;
        if (fread(r->raw, (size_t)rb, (size_t)want, r->f) != (size_t)want) return -1;
        for (long long i = 0; i < want; ++i) {
            if (r->raw[i * (r->d + 1)] != r->d) return -1;   /* a row of another dimension */
            memcpy(dst + i * r->d, r->raw + i * (r->d + 1) + 1, (size_t)r->d * sizeof(float));
        }
        dst += want * r->d;
        rows -= want;
        r->next += want;
    }
    return 0;
}

int main(int argc, const char* argv[]) {
    if (argc < 4) {
        fprintf(stderr, "Usage: %s <input file> <output template> <m> [--num-threads <nt>] "
                        "[--compute-error] [--kmeans-iterations n] [--centroids f]\n", argv[0]);
        return 1;
    }
    const char* input = argv[1];
    const char* tmpl = argv[2];
    int m = atoi(argv[3]);
    int compute_error = 0, iters = 10, k = 256;
    const char* cfile = NULL;
    for (int i = 4; i < argc; ++i) {
        if (!strcmp(argv[i], "--num-threads") && i + 1 < argc) ++i;
        else if (!strcmp(argv[i], "--compute-error")) compute_error = 1;
        else if (!strcmp(argv[i], "--kmeans-iterations") && i + 1 < argc) iters = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--centroids") && i + 1 < argc) cfile = argv[++i];
        else if (!strcmp(argv[i], "--seed") && i + 1 < argc) rng_state = strtoull(argv[++i], NULL, 10) | 1;
        else {
            fprintf(stderr, "Unknown argument: %s\n", argv[i]);
            return 1;
        }
    }
    long long n = 0;
    int d = 0;
    if (fvecs_load_meta(input, &n, &d) || m <= 0 || d % m) {
        fprintf(stderr, "cannot read %s or D %% m != 0\n", input);
        return 1;
    }
    const int ds = d / m;
    unsigned char* codes = (unsigned char*)malloc((size_t)n * m + 1);
    /* every pass streams the file (the reference reads 128K-row batches, pq_encoder.c:58-80,
     * 89-113): the input is never held whole, on the host or on the device */
    fvecs_reader_t rd = {fopen(input, "rb"), d, NULL, 1 << 16, 0};
    rd.raw = (int32_t*)malloc((size_t)rd.cap * (d + 1) * 4);
    if (!rd.f || !rd.raw || !codes) {
        fprintf(stderr, "cannot read %s\n", input);
        return 1;
    }
    centroids_codebook_t cb;
    if (cfile) {
        if (centroids_codebook_load(&cb, cfile, m, k) || cb.num_dimensions != ds) {
            fprintf(stderr, "bad centroids file %s\n", cfile);
            return 1;
        }
    } else {
        /* seeded init: k rows drawn from the file, then GPU Lloyd with fixed-point means */
        centroids_codebook_init(&cb, m, k, ds);
        float* row = (float*)malloc((size_t)d * sizeof(float));
        for (int c = 0; c < k; ++c) {
            long long v = n ? (long long)(rng_next() % (unsigned long long)n) : 0;
            if (n && fvecs_rows(&rd, v, 1, row)) {
                fprintf(stderr, "cannot read %s\n", input);
                return 1;
            }
            for (int i = 0; i < m; ++i)
                memcpy(cb.centroids[i] + (size_t)c * ds, n ? row + (long long)i * ds : row,
                       n ? ds * sizeof(float) : 0);
        }
        free(row);
        int trc = pq_train_rows(&cb, d, n, fvecs_rows, &rd, iters, 0);
        if (trc) {
            fprintf(stderr, "pq_train failed: %d\n", trc);
            return 1;
        }
    }
    int rc = pq_encode_rows(&cb, d, n, fvecs_rows, &rd, codes, 0);
    if (rc) {
        fprintf(stderr, "pq_encode failed: %d\n", rc);
        return 1;
    }
    char* pc = concat(tmpl, "pq_centroids.fvecsl");
    char* pi = concat(tmpl, "pq_indices.bvecsl");
    if (centroids_codebook_save(&cb, pc)) {
        fprintf(stderr, "cannot write %s\n", pc);
        return 1;
    }
    FILE* f = fopen(pi, "wb");
    if (!f) {
        fprintf(stderr, "cannot open %s\n", pi);
        return 1;
    }
    save_vecs_light_meta_file(f, n, m);
    const size_t wrote = n ? fwrite(codes, (size_t)m, (size_t)n, f) : 0;
    if (wrote != (size_t)n || ferror(f) || fclose(f)) {
        fprintf(stderr, "cannot write %s\n", pi);
        return 1;
    }
    if (compute_error) {
        double err = 0;
        if (pq_compute_error_rows(&cb, d, n, fvecs_rows, &rd, codes, 0, &err)) {
            fprintf(stderr, "compute_error failed\n");
            return 1;
        }
        char* pe = concat(tmpl, "pq_error");
        FILE* ef = fopen(pe, "a");
        if (!ef || fprintf(ef, "%lf\n", err) < 0 || fclose(ef)) {
            fprintf(stderr, "cannot write %s\n", pe);
            return 1;
        }
        free(pe);
    }
    free(pc);
    free(pi);
    centroids_codebook_destroy(&cb);
    free(codes);
    fclose(rd.f);
    free(rd.raw);
    return 0;
}
