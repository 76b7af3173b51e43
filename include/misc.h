/*
 * misc.h -- pq_huffman_amd drop-in for the reference's src/misc.h (misc.h:1-26).
 * Same types and function signatures; implemented in pq_huffman_amd/csrc/host/misc.c.
 */
#ifndef _HUFFMAN_MISC_H
#define _HUFFMAN_MISC_H

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned int vector_id_t;          /* misc.h:4 */
typedef unsigned char byte_t;              /* misc.h:24 */

int imin(int a, int b);
long long iminll(long long a, long long b);
long long iclampll(long long value, long long min_value, long long max_value);

/* NOTE: allocates with malloc (misc.h:11) */
char* concat(const char* prefix, const char* suffix);

long long load_num_elements(const char* filename, long long element_size);

#define MS 1000

#ifdef __cplusplus
}
#endif

#endif /* _HUFFMAN_MISC_H */
