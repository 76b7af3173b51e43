/* pq.c -- the library part of pq_encoder.c the reference never extracted (pq.h is empty
 * there): centroids_codebook_t (pq_encoder.c:34-40, :227-255) and .fvecs reading
 * (pq_encoder.c:46-80, here in one pass instead of one pass per subspace). */
#include "pq.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "vecs_io.h"

void centroids_codebook_init(centroids_codebook_t* cb, int num_parts, int num_clusters,
                             int num_dimensions) {
    cb->num_parts = num_parts;
    cb->num_clusters = num_clusters;
    cb->num_dimensions = num_dimensions;
    cb->centroids_pool = (float*)calloc((size_t)num_parts * num_clusters * num_dimensions, sizeof(float));
    cb->centroids = (float**)malloc(sizeof(float*) * (num_parts > 0 ? num_parts : 1));
    for (int i = 0; i < num_parts; ++i)
        cb->centroids[i] = cb->centroids_pool + (size_t)i * num_clusters * num_dimensions;
}

void centroids_codebook_destroy(centroids_codebook_t* cb) {
    free(cb->centroids_pool);
    free(cb->centroids);
    cb->centroids_pool = NULL;
    cb->centroids = NULL;
}

int centroids_codebook_save(const centroids_codebook_t* cb, const char* filename) {
    FILE* f = fopen(filename, "wb");
    if (!f) return -1;
    save_vecs_light_meta_file(f, (long long)cb->num_parts * cb->num_clusters, cb->num_dimensions);
    size_t cnt = (size_t)cb->num_parts * cb->num_clusters * cb->num_dimensions;
    size_t w = fwrite(cb->centroids_pool, sizeof(float), cnt, f);
    const int bad = ferror(f);
    return fclose(f) == 0 && !bad && w == cnt ? 0 : -1;
}

int centroids_codebook_load(centroids_codebook_t* cb, const char* filename, int num_parts,
                            int num_clusters) {
    long long rows = 0;
    int dsub = 0;
    float* data = (float*)load_vecs_light_filename(filename, sizeof(float), &rows, &dsub);
    if (!data) return -1;
    if (num_parts <= 0 && num_clusters > 0) num_parts = (int)(rows / num_clusters);
    if (num_clusters <= 0 && num_parts > 0) num_clusters = (int)(rows / num_parts);
    if (num_parts <= 0 || num_clusters <= 0 || (long long)num_parts * num_clusters != rows) {
        free(data);
        return -1;
    }
    cb->num_parts = num_parts;
    cb->num_clusters = num_clusters;
    cb->num_dimensions = dsub;
    cb->centroids_pool = data;
    cb->centroids = (float**)malloc(sizeof(float*) * num_parts);
    for (int i = 0; i < num_parts; ++i) cb->centroids[i] = data + (size_t)i * num_clusters * dsub;
    return 0;
}

int fvecs_load_meta(const char* filename, long long* num_vectors, int* num_dimensions) {
    FILE* f = fopen(filename, "rb");
    if (!f) return -1;
    int32_t d = 0;
    if (fread(&d, 4, 1, f) != 1 || d <= 0) {
        fclose(f);
        return -1;
    }
    fseek(f, 0, SEEK_END);
    long long size = ftell(f);
    fclose(f);
    long long row = 4LL + 4LL * d;
    if (size % row) return -1;
    *num_vectors = size / row;
    *num_dimensions = d;
    return 0;
}

float* fvecs_load(const char* filename, long long* num_vectors, int* num_dimensions) {
    long long n = 0;
    int d = 0;
    if (fvecs_load_meta(filename, &n, &d)) return NULL;
    FILE* f = fopen(filename, "rb");
    float* out = (float*)malloc((size_t)(n > 0 ? n : 1) * d * sizeof(float));
    const long long batch = 1 << 16;
    float* rows = (float*)malloc((size_t)batch * (d + 1) * sizeof(float));
    for (long long got = 0; got < n;) {
        long long want = n - got < batch ? n - got : batch;
        size_t r = fread(rows, (size_t)(d + 1) * sizeof(float), (size_t)want, f);
        if (r == 0) break;
        for (size_t i = 0; i < r; ++i)
            for (int j = 0; j < d; ++j) out[(got + (long long)i) * d + j] = rows[i * (d + 1) + 1 + j];
        got += (long long)r;
    }
    free(rows);
    fclose(f);
    *num_vectors = n;
    *num_dimensions = d;
    return out;
}
