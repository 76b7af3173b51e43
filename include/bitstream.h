/*
 * bitstream.h -- drop-in for the reference's src/bitstream.h:8-22 (bit_stream_t API).
 * MSB-first within bytes, zero pad to a byte on destroy of a write stream.
 * Replaces: bitstream.c:27-194.  Implemented in csrc/host/bitstream.c (word-at-a-time,
 * byte-identical output).
 */
#ifndef _BITSTREAM_H
#define _BITSTREAM_H

#include <stdio.h>

#include "misc.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    BYTE_NUM_BITS = sizeof(byte_t) * 8
};

typedef struct _bit_stream bit_stream_t;

bit_stream_t* bit_stream_create_from_file(FILE* file);
bit_stream_t* bit_stream_create_from_file_buffered(FILE* file, long long buffer_size_bytes);
bit_stream_t* bit_stream_destroy(bit_stream_t* stream);                 /* always NULL */
bit_stream_t* bit_stream_destroy_file(bit_stream_t* stream, int close_file); /* always NULL */

int bit_stream_flush(bit_stream_t* stream, int add_pad);
int bit_stream_write(bit_stream_t* stream, const byte_t* data, long long bit_length);
void bit_stream_read(bit_stream_t* stream, byte_t* data, long long bit_length);
int bit_stream_read_bit(bit_stream_t* stream);

#ifdef __cplusplus
}
#endif

#endif /* _BITSTREAM_H */
