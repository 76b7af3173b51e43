/*
 * ref_knn_harness.c -- TEST INFRASTRUCTURE ONLY (oracle side, never shipped, never linked
 * by pq_huffman_amd).
 *
 * A thin driver compiled TOGETHER WITH the reference's own sources
 * /root/reference/src/{fast_nn_blocks_info,fast_nn_temp_file,fast_nn_block,misc,vecs_io}.c
 * by oracle/ref.mk into oracle/_ref/libref_knn.so, so the parts of compute_nn_fast that do
 * not need yael can pin the oracle (tests/golden/forest_*.npz, oracle/gen_golden.py):
 *   refk_blocks_info  blocks_info_init over an .fvecs file (fast_nn_blocks_info.c:94-112)
 *   refk_in_block     is_vector_in_block (:187-193) on a blocks_info_t built from arrays
 *   refk_merge        init_empty_batch_for_temp_file + fast_nn_heap_push in the given order
 *                     + fast_nn_heap_sort (fast_nn_temp_file.c:48-63,93-108)
 * Nothing here re-implements an algorithm: every value comes from the reference functions.
 */
#include <stdlib.h>
#include <string.h>

#include "fast_nn_blocks_info.h"
#include "fast_nn_temp_file.h"

int refk_blocks_info(const char* fvecs, long long n, int d, int ns, int nb, double overlap,
                     float* starts, float* ends) {
    blocks_info_t bi;
    blocks_info_init(&bi, fvecs, n, d, ns, nb, overlap);
    for (int i = 0; i < ns; ++i) {
        memcpy(starts + i * nb, bi.dimension_infos[i].block_starts, sizeof(float) * nb);
        memcpy(ends + i * nb, bi.dimension_infos[i].block_ends, sizeof(float) * nb);
    }
    const long long total = bi.num_blocks_total;
    blocks_info_destroy(&bi);
    return (int)total;
}

int refk_in_block(const float* vec, int d, int ns, int nb, const float* starts,
                  const float* ends, long long block) {
    blocks_info_t bi;
    bi.num_dimensions = ns;
    bi.block_overlap_fraction = 0.0;
    bi.num_blocks_per_dim = nb;
    bi.num_blocks_total = 1;
    bi.dimension_infos = malloc(sizeof(*bi.dimension_infos) * ns);
    for (int i = 0; i < ns; ++i) {
        block_dimension_info_t* di = bi.dimension_infos + i;
        di->dimension = ns - 1 - i;   /* blocks_info_init's order (:106) */
        di->num_blocks = nb;
        di->block_id_mask = 1;
        for (int q = 0; q < di->dimension; ++q) di->block_id_mask *= nb;
        di->block_starts = (float*)starts + i * nb;
        di->block_ends = (float*)ends + i * nb;
        bi.num_blocks_total *= nb;
    }
    const int r = is_vector_in_block(vec, d, &bi, block);
    free(bi.dimension_infos);
    return r;
}

void refk_merge(long long n, int num_nn, long long npush, const long long* rows,
                const unsigned* idx, const float* dist, unsigned* out_idx, float* out_dist) {
    nn_item_t* heaps = malloc(sizeof(nn_item_t) * num_nn * (n ? n : 1));
    init_empty_batch_for_temp_file(heaps, num_nn, n);
    for (long long q = 0; q < npush; ++q) {
        nn_item_t it;
        it.index = idx[q];
        it.dist = dist[q];
        fast_nn_heap_push(heaps + rows[q] * num_nn, &it, num_nn);
    }
    for (long long v = 0; v < n; ++v)
        fast_nn_heap_sort(heaps + v * num_nn, num_nn, out_idx + v * num_nn, out_dist + v * num_nn);
    free(heaps);
}
