/* pq_encoder -- CLI-compatible replacement for the reference's src/pq_encoder.c
 * (usage pq_encoder.c:121-175; outputs :207-213, :248-255, :290-295).
 *   pq_encoder <input.fvecs> <output template> <m> [--num-threads t] [--compute-error]
 *              [--kmeans-iterations n] [--centroids <pq_centroids.fvecsl>] [--seed s]
 * Assignment and training run on the GPU (libpqh).  Training: deterministic Lloyd
 * iterations on the GPU (pq_train: exact assignment, fixed-point centroid means) from a
 * seeded sample init (yael's time-seeded Berkeley init is not reproducible); --centroids
 * skips training.  --num-threads is accepted for compatibility. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
    float* x = fvecs_load(input, &n, &d);
    if (!x || m <= 0 || d % m) {
        fprintf(stderr, "cannot read %s or D %% m != 0\n", input);
        return 1;
    }
    const int ds = d / m;
    unsigned char* codes = (unsigned char*)malloc((size_t)n * m + 1);
    centroids_codebook_t cb;
    if (cfile) {
        if (centroids_codebook_load(&cb, cfile, m, k) || cb.num_dimensions != ds) {
            fprintf(stderr, "bad centroids file %s\n", cfile);
            return 1;
        }
    } else {
        centroids_codebook_init(&cb, m, k, ds);
        for (int c = 0; c < k; ++c) {
            long long v = n ? (long long)(rng_next() % (unsigned long long)n) : 0;
            for (int i = 0; i < m; ++i)
                memcpy(cb.centroids[i] + (size_t)c * ds, x + v * d + (long long)i * ds, ds * sizeof(float));
        }
        int trc = pq_train(&cb, x, n, d, iters);   /* GPU Lloyd, fixed-point means */
        if (trc) {
            fprintf(stderr, "pq_train failed: %d\n", trc);
            return 1;
        }
    }
    int rc = pq_encode(&cb, x, n, d, codes);
    if (rc) {
        fprintf(stderr, "pq_encode failed: %d\n", rc);
        return 1;
    }
    char* pc = concat(tmpl, "pq_centroids.fvecsl");
    char* pi = concat(tmpl, "pq_indices.bvecsl");
    centroids_codebook_save(&cb, pc);
    FILE* f = fopen(pi, "wb");
    save_vecs_light_meta_file(f, n, m);
    fwrite(codes, (size_t)m, (size_t)n, f);
    fclose(f);
    if (compute_error) {
        double err = 0;
        if (pq_compute_error(&cb, x, n, d, codes, &err) == 0) {
            char* pe = concat(tmpl, "pq_error");
            FILE* ef = fopen(pe, "a");
            fprintf(ef, "%lf\n", err);
            fclose(ef);
            free(pe);
        }
    }
    free(pc);
    free(pi);
    centroids_codebook_destroy(&cb);
    free(codes);
    free(x);
    return 0;
}
