/*
 * vecs_io.h -- drop-in for the reference's src/vecs_io.h:8-20: light ".xvecsl" files,
 * header u32 N, u32 D, then N*D raw elements (vecs_io.c:16-76).  N is 32-bit on disk
 * (vecs_io.c:45), so N < 2^32.
 */
#ifndef _VECS_IO_H
#define _VECS_IO_H

#include <stddef.h>
#include <stdio.h>

#include "misc.h"

#ifdef __cplusplus
extern "C" {
#endif

byte_t* load_vecs_light_filename(const char* filename, size_t element_size,
                                 long long* num_elements_out, int* num_dimensions_out);
byte_t* load_vecs_light_file(FILE* file, size_t element_size,
                             long long* num_elements_out, int* num_dimensions_out);

void load_vecs_light_meta_filename(const char* filename, long long* num_elements_out,
                                   int* num_dimensions_out);
void load_vecs_light_meta_file(FILE* file, long long* num_elements_out,
                               int* num_dimensions_out);
long long load_vecs_num_vectors_filename(const char* filename);
int load_vecs_num_dimensions_filename(const char* filename);

void save_vecs_light_meta_file(FILE* file, long long num_elements, int num_dimensions);

#ifdef __cplusplus
}
#endif

#endif /* _VECS_IO_H */
