/* fast_nn_block.c -- drop-in for the reference's src/fast_nn_block.c:6-71 (block_t).
 * Same observable behaviour: initial_capacity is ignored and every block starts with room
 * for 100 rows (fast_nn_block.c:11); growth is (capacity + 1) * 2 (:41-44). */
#include "fast_nn_block.h"

#include <stdlib.h>
#include <string.h>

void block_init(block_t* block, long long block_id, int num_dimensions, long long initial_capacity,
                int init_flags) {
    block->id = block_id;
    block->num_dimensions = num_dimensions;
    (void)initial_capacity;   /* ignored, as in the reference */
    block->capacity = 100;
    block->size = 0;
    block->data = (init_flags & BLOCK_INIT_WITH_DATA)
                      ? (float*)malloc(sizeof(float) * num_dimensions * block->capacity)
                      : NULL;
    block->indices = (init_flags & BLOCK_INIT_WITH_INDICES)
                         ? (long long*)malloc(sizeof(long long) * block->capacity)
                         : NULL;
}

void block_destroy(block_t* block) {
    free(block->data);
    free(block->indices);
    block->data = NULL;
    block->indices = NULL;
    block->id = -1;
    block->num_dimensions = 0;
    block->capacity = 0;
    block->size = 0;
}

void block_realloc(block_t* block, long long new_capacity) {
    if (block->data)
        block->data = (float*)realloc(block->data, sizeof(float) * block->num_dimensions * new_capacity);
    if (block->indices)
        block->indices = (long long*)realloc(block->indices, sizeof(long long) * new_capacity);
    block->capacity = new_capacity;
}

void block_push(block_t* block, long long index, const float* vector) {
    if (block->size >= block->capacity) block_realloc(block, (block->capacity + 1) * 2);
    if (block->indices) block->indices[block->size] = index;
    if (block->data)
        memcpy(block->data + block->size * block->num_dimensions, vector,
               sizeof(float) * block->num_dimensions);
    ++block->size;
}

void block_set_id(block_t* block, long long block_id) {
    block->id = block_id;
    block->size = 0;
}
