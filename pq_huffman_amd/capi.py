"""ctypes binding of libpqh.so -- the C ABI declared in include/*.h.

The library is built in-tree (pq_huffman_amd/lib/libpqh.so, `python -m pq_huffman_amd.build`
or __graft_entry__.build()).  Loading fails loudly when it is missing: there is no Python
or CPU fallback for any GPU entry point.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libpqh.so")
# diagnostics only: an alternative in-tree build of the same library (tools/ A/B runs)
LIB_PATH = os.environ.get("PQH_LIB", LIB_PATH)

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
ULL = ctypes.c_ulonglong
D = ctypes.c_double
S = ctypes.c_char_p

PQH_OK = 0
STATUS = {0: "ok", -1: "invalid argument", -2: "no HIP device", -3: "HIP runtime error",
          -4: "unsupported configuration", -5: "code longer than 56 bits", -6: "corrupt stream",
          -7: "out of memory", -8: "output buffer too small",
          -9: "another rank's part of the sharded call failed",
          -10: "a collective hook failed"}


class PqhError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {STATUS.get(status, status)} ({status})")


class HuffmanCodeItem(ctypes.Structure):          # huffman.h huffman_code_item_t
    _fields_ = [("code", ctypes.POINTER(ctypes.c_ubyte)), ("bit_length", I)]


class HuffmanCodebook(ctypes.Structure):          # huffman.h huffman_codebook_t
    _fields_ = [("codefield", ctypes.POINTER(ctypes.c_ubyte)), ("alphabet_size", I),
                ("is_context", I), ("num_items", I), ("items", ctypes.POINTER(HuffmanCodeItem))]


class HuffmanStats(ctypes.Structure):             # stats.h huffman_stats_t
    _fields_ = [("num_vectors", LL), ("m", I), ("k_star", I), ("sum_length", D),
                ("partial_lengths", ctypes.POINTER(D)), ("num_roots", I)]


class Block(ctypes.Structure):                    # fast_nn_block.h block_t
    _fields_ = [("id", ctypes.c_longlong), ("num_dimensions", ctypes.c_int),
                ("capacity", ctypes.c_longlong), ("indices", ctypes.POINTER(ctypes.c_longlong)),
                ("data", ctypes.POINTER(ctypes.c_float)), ("size", ctypes.c_longlong)]


# pqh.h pqh_shard_comm_t: collective hooks over device buffers
ALL_REDUCE_U32 = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_longlong, ctypes.c_void_p)
ALL_GATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_longlong, ctypes.c_void_p)


class ShardComm(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("world", ctypes.c_int), ("rank", ctypes.c_int),
                ("all_reduce_sum_u32", ALL_REDUCE_U32), ("all_gather", ALL_GATHER)]


class EncodeOptions(ctypes.Structure):            # pqh.h pqh_encode_options_t
    _fields_ = [("context", I), ("sort", I), ("chunk_vectors", I), ("only_estimate", I)]


# (name, restype, argtypes) of every function the headers declare
SIGNATURES = [
    # misc.h
    ("imin", I, [I, I]), ("iminll", LL, [LL, LL]), ("iclampll", LL, [LL, LL, LL]),
    ("concat", P, [S, S]), ("load_num_elements", LL, [S, LL]),
    # bitstream.h
    ("bit_stream_create_from_file", P, [P]), ("bit_stream_create_from_file_buffered", P, [P, LL]),
    ("bit_stream_destroy", P, [P]), ("bit_stream_destroy_file", P, [P, I]),
    ("bit_stream_flush", I, [P, I]), ("bit_stream_write", I, [P, P, LL]),
    ("bit_stream_read", None, [P, P, LL]), ("bit_stream_read_bit", I, [P]),
    # huffman.h
    ("huffman_dump_code", None, [P, P]), ("huffman_codebook_dump", None, [P, P]),
    ("huffman_counts_context_dump", None, [P, I, P]),
    ("huffman_codebook_save", None, [P, P]), ("huffman_codebook_load", None, [P, P]),
    ("huffman_codebook_encode_init", None, [P, I, P]),
    ("huffman_codebook_context_encode_init", None, [P, I, P]),
    ("huffman_codebook_destroy", None, [P]), ("huffman_estimate_size", D, [P, P]),
    ("huffman_decoder_create", P, [P]), ("huffman_decoder_destroy", P, [P]),
    ("huffman_decoder_reset", None, [P]), ("huffman_decoder_set_prev_symbol", None, [P, I]),
    ("huffman_decoder_push_bit", I, [P, I]), ("huffman_decoder_push_bits", I, [P, P, I]),
    ("huffman_decoder_read_symbol", I, [P, P]),
    # vecs_io.h
    ("load_vecs_light_filename", P, [S, ctypes.c_size_t, P, P]),
    ("load_vecs_light_file", P, [P, ctypes.c_size_t, P, P]),
    ("load_vecs_light_meta_filename", None, [S, P, P]),
    ("load_vecs_light_meta_file", None, [P, P, P]),
    ("load_vecs_num_vectors_filename", LL, [S]), ("load_vecs_num_dimensions_filename", I, [S]),
    ("save_vecs_light_meta_file", None, [P, LL, I]),
    # stats.h
    ("huffman_stats_init", None, [P, LL, I, I]), ("huffman_stats_destroy", None, [P]),
    ("huffman_stats_push", None, [P, I, D]), ("huffman_stats_print", None, [P]),
    ("huffman_stats_print_filename", None, [P, S]), ("huffman_stats_print_file", None, [P, P]),
    # fast_nn_block.h
    ("block_init", None, [P, LL, I, LL, I]), ("block_destroy", None, [P]),
    ("block_push", None, [P, LL, P]), ("block_realloc", None, [P, LL]),
    ("block_set_id", None, [P, LL]),
    # pq.h
    ("centroids_codebook_init", None, [P, I, I, I]), ("centroids_codebook_destroy", None, [P]),
    ("centroids_codebook_save", I, [P, S]), ("centroids_codebook_load", I, [P, S, I, I]),
    ("fvecs_load_meta", I, [S, P, P]), ("fvecs_load", P, [S, P, P]),
    ("pq_encode", I, [P, P, LL, I, P]), ("pq_compute_error", I, [P, P, LL, I, P, P]),
    ("pq_train", I, [P, P, LL, I, I]), ("pq_encode_rows", I, [P, I, LL, P, P, P, LL]),
    ("pq_train_rows", I, [P, I, LL, P, P, I, LL]),
    ("pq_compute_error_rows", I, [P, I, LL, P, P, P, LL, P]),
    # pqh.h
    ("pqh_ctx_create", I, [P, I]), ("pqh_ctx_destroy", I, [P]), ("pqh_ctx_set_stream", I, [P, P]),
    ("pqh_ctx_create_cu_limited", I, [P, I, I]), ("pqh_ctx_create_cu_split", I, [P, I, I, I]), ("pqh_ctx_stream", P, [P]),
    ("pqh_ctx_sync", I, [P]), ("pqh_ctx_release_scratch", I, [P]), ("pqh_status_string", S, [I]), ("pqh_ctx_last_error", S, [P]),
    ("pqh_device_count", I, [P]),
    ("pqh_pq_create", I, [P, P, I, I, I, P]), ("pqh_pq_destroy", I, [P]),
    ("pqh_pq_assign", I, [P, P, P, LL, LL, P, P, I]),
    ("pqh_pq_assign_parts", I, [P, P, P, LL, LL, P, LL, P, I]),
    ("pqh_pq_last_rerank_count", I, [P, P]),
    ("pqh_pq_error", I, [P, P, P, LL, LL, P, P]),
    ("pqh_pq_reconstruct", I, [P, P, P, LL, P, LL]),
    ("pqh_kmeans_train", I, [P, P, LL, LL, I, I, I, I, P]),
    ("pqh_histogram", I, [P, P, LL, I, I, I, P, P]),
    ("pqh_histogram_set", I, [P, P, LL, I, I, I, P, P]),
    ("pqh_histogram_parts", I, [P, P, LL, LL, I, I, I, P, P, I]),
    ("pqh_histogram_partial_parts", I, [P, P, LL, LL, I, I, P, P]),
    ("pqh_histogram_partial_bytes", LL, [LL, I, I]),
    ("pqh_histogram_partial", I, [P, P, LL, I, I, P, P]),
    ("pqh_histogram_reduce", I, [P, P, LL, I, I, P, I]),
    ("pqh_tables_create", I, [P, P, I, P]), ("pqh_tables_destroy", I, [P]),
    ("pqh_tables_alloc", I, [P, I, I, I, P]), ("pqh_tables_build", I, [P, P, P]),
    ("pqh_tables_build_impl", I, [P, P, P, I]),
    ("pqh_tables_build_trees", I, [P, P, P, I]), ("pqh_tables_build_luts", I, [P, P]),
    ("pqh_tables_encode_ready", I, [P]),
    ("pqh_tables_build_pair", I, [P, P, P, P, P]),
    ("pqh_tables_upload", I, [P, P, P]), ("pqh_tables_status", I, [P, P]),
    ("pqh_tables_codebooks", I, [P, P, P]),
    ("pqh_codebooks_build", I, [P, I, I, I, P, I]),
    ("pqh_encode_size", I, [P, P, P, LL, I, P, P]),
    ("pqh_encode_write", I, [P, P, P, LL, I, P, ULL, P, ULL, I, P, P, P]),
    ("pqh_encode_write_at", I, [P, P, P, LL, I, P, P, P, ULL, I, P, P, P]),
    ("pqh_encode_write_parts", I, [P, P, P, LL, LL, I, P, ULL, P, ULL, I, P, P, P]),
    ("pqh_transpose_codes", I, [P, P, LL, LL, I, I, P]),
    ("pqh_decode", I, [P, P, P, ULL, LL, I, I, P, P, P]),
    ("pqh_decode_status", I, [P]), ("pqh_encode_status", I, [P]),
    ("pqh_chunk_index_host", I, [P, P, ULL, LL, I, I, P, P]),
    ("pqh_sort_rows", I, [P, P, LL, I, P]),
    ("pqh_shard_block", I, [LL, I, I, P]), ("pqh_shard_scratch_bytes", LL, [I, I]),
    ("pqh_shard_encode", I, [P, P, P, P, I, I, I, P, P, P, ULL, I, P, P, P, P, P]),
    ("pqh_shard_status", I, [P, P]),
    ("pqh_shard_encode_tables", I, [P, P, P, P, I, I, I, P, P, P]),
    ("pqh_shard_encode_write", I, [P, P, P, P, I, I, I, P, P, ULL, I, P, P, P, P, I, P]),
    ("pqh_shard_encode_tables_parts", I, [P, P, P, P, LL, I, I, I, P, P, P, P]),
    ("pqh_shard_encode_write_parts", I, [P, P, P, P, LL, I, I, I, P, P, ULL, I, P, P, P, P, I, P]),
    ("pqh_shard_offsets", I, [P, I, I, P, P]),
    ("pqh_shard_stitch", I, [I, P, P, P, P, ULL]),
    ("pqh_shard_halo_source", I, [P, I, I, P, P]),
    ("pqh_debug_poison_lds", I, [P, ctypes.c_uint]),
    ("pqh_ctx_set_tuning", I, [P, I, D]),
    ("pqh_tree_order", I, [LL, LL, P, P, P, P, P]),
    ("pqh_tree_order_device", I, [P, LL, LL, P, P, P, P, P, P]),
    ("pqh_tree_ext_index_device", LL, [P, LL, P, I, I, P, P, P]),
    ("pqh_tree_gather", I, [P, P, LL, I, I, P, P, P, P]),
    ("pqh_tree_status", I, [P]),
    ("pqh_histogram_tree", I, [P, P, P, LL, I, I, P]),
    ("pqh_encode_tree_write", I, [P, P, P, P, LL, ULL, P, ULL, I, P, P]),
    ("pqh_tree_ext_index", LL, [LL, P, I, P, P, P]),
    ("pqh_decode_tree", I, [P, P, P, ULL, LL, I, P, P, P, P, P]),
    ("pqh_encode_tree_files", I, [P, LL, I, I, S, S]),
    ("pqh_decode_tree_files", I, [S, P, P, P]),
    ("pqh_encode_files", I, [P, LL, I, P, S]),
    ("pqh_decode_files", I, [S, P, P, P]),
    ("pqh_knn_blocks_info", I, [P, P, LL, LL, I, I, I, D, P, P]),
    ("pqh_knn_fast", I, [P, P, LL, LL, I, I, I, I, P, P, P, P, P]),
    ("pqh_mst_build", I, [P, P, P, LL, I, I, P, I, ctypes.c_float, P, P, P]),
    ("pqh_knn_fast_files", I, [S, S, I, P]),
    ("pqh_mst_files", I, [S, S, I, S, ctypes.c_float]),
]

_lib = None


def lib():
    """Load libpqh.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `python -m pq_huffman_amd.build`"
                               " (the HIP extension is required; there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status: int, what: str = "pqh") -> None:
    if status != PQH_OK:
        raise PqhError(status, what)
