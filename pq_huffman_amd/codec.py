"""Python mirror of the reference's encode/decode flow over the pqh C ABI.

The reference pipeline is pq_encoder -> huffman_encoder ->
huffman_decoder, gluing CLI programs through files.  Here the same stages run as C-ABI
calls on device-resident data:

    PQ.assign            pq_encoder.c:270-272 (yael kmeans assignment) + :192-205
    kmeans_train         pq_encoder.c:265-274 (training, deterministic Lloyd on the GPU)
    sort_rows            huffman_encoder.c:301-317 (default sort mode)
    histogram            huffman_encoder.c:139-205
    build_codebooks      huffman_encoder.c:377-388 (huffman_codebook_[context_]encode_init)
    encode               huffman_encoder.c:413-428 (+ sidecar chunk index)
    decode               huffman_decoder.c:206-255

torch is used only for device memory and the stream (data_ptr / cuda_stream); every
computation is a libpqh kernel.  Device buffers are torch tensors owned by the caller.
"""
from __future__ import annotations

import ctypes
import os
import tempfile
from dataclasses import dataclass

import numpy as np

from .capi import (EncodeOptions, HuffmanCodebook, PqhError, check, lib)

_libc = ctypes.CDLL(None)
_libc.fopen.restype = ctypes.c_void_p
_libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
_libc.fclose.argtypes = [ctypes.c_void_p]
_libc.fwrite.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
_libc.fseek.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int]


def _ptr(t):
    """device/host pointer of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(t.data_ptr())


def _torch():
    import torch
    return torch


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().pqh_device_count(ctypes.byref(n))
    return n.value


class Context:
    """pqh_ctx_t bound to a torch device and a stream (pqh.h).

    Default: torch's current stream, so torch's fills and copies are ordered with the pqh
    kernels.  cus > 0: the context keeps its own stream limited to that many compute units
    (pqh_ctx_create_cu_split), or with complement=True to all the OTHER compute units;
    `stream` is then a torch.cuda.ExternalStream over it."""

    def __init__(self, device: int = 0, stream=None, cus: int = 0, complement: bool = False):
        torch = _torch()
        self.device = device
        torch.cuda.set_device(device)
        self.ptr = ctypes.c_void_p()
        if cus != 0:   # (< 0: all CUs on a CU-masked stream, a hardware queue of its own)
            check(lib().pqh_ctx_create_cu_split(ctypes.byref(self.ptr), device, cus,
                                                int(complement)), "pqh_ctx_create_cu_split")
            self.stream = torch.cuda.ExternalStream(lib().pqh_ctx_stream(self.ptr), device=device)
            return
        self.stream = stream or torch.cuda.current_stream(device)
        check(lib().pqh_ctx_create(ctypes.byref(self.ptr), device), "pqh_ctx_create")
        # bind to torch's stream (often the NULL/default stream) so torch's allocations,
        # fills and copies are ordered with the pqh kernels
        check(lib().pqh_ctx_set_stream(self.ptr, ctypes.c_void_p(self.stream.cuda_stream)),
              "pqh_ctx_set_stream")

    def set_stream(self, stream) -> None:
        self.stream = stream
        check(lib().pqh_ctx_set_stream(self.ptr, ctypes.c_void_p(stream.cuda_stream)))

    TUNE = {"assign_wgs_per_cu": 1, "hist_split": 2, "hist_block": 3, "enc_impl": 4}

    def set_tuning(self, **kw) -> "Context":
        """launch shapes of this context's kernels (pqh_ctx_set_tuning; results never
        change): assign_wgs_per_cu, hist_split, hist_block, enc_impl (1 tiled, 2 one-pass)
        -- 0 restores the default"""
        for key, value in kw.items():
            check(lib().pqh_ctx_set_tuning(self.ptr, self.TUNE[key], float(value)),
                  f"pqh_ctx_set_tuning({key})")
        return self

    def sync(self) -> None:
        check(lib().pqh_ctx_sync(self.ptr), "pqh_ctx_sync")

    def release_scratch(self) -> None:
        """free the context's grow-only device scratch (pqh_ctx_release_scratch)"""
        check(lib().pqh_ctx_release_scratch(self.ptr), "pqh_ctx_release_scratch")

    def last_error(self) -> str:
        return (lib().pqh_ctx_last_error(self.ptr) or b"").decode()

    def close(self) -> None:
        if self.ptr:
            lib().pqh_ctx_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PQ:
    """Prepared sub-codebooks on the device (pq.h centroids_codebook_t + MFMA fragments)."""

    def __init__(self, ctx: Context, centroids: np.ndarray):
        c = np.ascontiguousarray(centroids, np.float32)
        self.m, self.k, self.dsub = c.shape
        self.ctx = ctx
        self.ptr = ctypes.c_void_p()
        check(lib().pqh_pq_create(ctx.ptr, _ptr(c), self.m, self.k, self.dsub,
                                  ctypes.byref(self.ptr)), "pqh_pq_create")

    @property
    def code_dtype(self):
        torch = _torch()
        return torch.uint8 if self.k <= 256 else torch.int16

    def assign(self, x, codes=None, counts=None, mode: int = 0, ctx: Context = None):
        """codes (n, m) of x; on `ctx`'s stream (any context of the same device, default the
        one the codebook was prepared with)."""
        torch = _torch()
        n = x.shape[0]
        if codes is None:
            codes = torch.empty((n, self.m), dtype=self.code_dtype, device=x.device)
        c = ctx or self.ctx
        check(lib().pqh_pq_assign(c.ptr, self.ptr, _ptr(x), n, x.stride(0), _ptr(codes),
                                  _ptr(counts), mode), "pqh_pq_assign")
        return codes

    def assign_parts(self, x, parts=None, counts=None, mode: int = 0, ctx: Context = None):
        """codes of x PART-MAJOR: parts (m, >= n), part i's codes contiguous in parts[i]
        (pqh_pq_assign_parts: the kernel stores whole lines)."""
        torch = _torch()
        n = x.shape[0]
        if parts is None:   # (rows padded to 128 codes: whole-line stores, see the kernel)
            parts = torch.empty((self.m, (n + 127) // 128 * 128), dtype=self.code_dtype,
                                device=x.device)[:, :n]
        c = ctx or self.ctx
        check(lib().pqh_pq_assign_parts(c.ptr, self.ptr, _ptr(x), n, x.stride(0), _ptr(parts),
                                        parts.stride(0), _ptr(counts), mode),
              "pqh_pq_assign_parts")
        return parts

    def rerank_count(self, ctx: Context = None) -> int:
        v = ctypes.c_ulonglong(0)
        check(lib().pqh_pq_last_rerank_count((ctx or self.ctx).ptr, ctypes.byref(v)))
        return v.value

    def error(self, x, codes) -> float:
        v = ctypes.c_double(0)
        check(lib().pqh_pq_error(self.ctx.ptr, self.ptr, _ptr(x), x.shape[0], x.stride(0),
                                 _ptr(codes), ctypes.byref(v)), "pqh_pq_error")
        return v.value

    def reconstruct(self, codes):
        torch = _torch()
        out = torch.empty((codes.shape[0], self.m * self.dsub), dtype=torch.float32,
                          device=codes.device)
        check(lib().pqh_pq_reconstruct(self.ctx.ptr, self.ptr, _ptr(codes), codes.shape[0],
                                       _ptr(out), out.stride(0)), "pqh_pq_reconstruct")
        return out

    def close(self):
        if self.ptr:
            lib().pqh_pq_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def kmeans_train(ctx: Context, x, init: np.ndarray, iters: int) -> np.ndarray:
    """Lloyd k-means of every subspace on the GPU (pqh_kmeans_train): exact assignment and
    fixed-point centroid means, deterministic; init [m][k][dsub] -> trained centroids."""
    cent = np.ascontiguousarray(init, np.float32).copy()
    m, k, ds = cent.shape
    check(lib().pqh_kmeans_train(ctx.ptr, _ptr(x), x.shape[0], x.stride(0), m, k, ds, iters,
                                 _ptr(cent)), "pqh_kmeans_train")
    return cent


class Codebooks:
    """m host codebooks (huffman.h huffman_codebook_t) built by the library."""

    def __init__(self, counts: np.ndarray, k: int, context: bool, threads: int = 0):
        counts = np.ascontiguousarray(counts, np.float64)
        self.m = counts.shape[0]
        self.k, self.context = k, bool(context)
        self.arr = (HuffmanCodebook * self.m)()
        check(lib().pqh_codebooks_build(_ptr(counts), self.m, k, int(context),
                                        ctypes.cast(self.arr, ctypes.c_void_p),
                                        threads or min(self.m, os.cpu_count() or 1)),
              "pqh_codebooks_build")
        self.counts = counts

    @classmethod
    def _empty(cls, m):
        obj = cls.__new__(cls)
        obj.m = m
        obj.arr = (HuffmanCodebook * m)()
        return obj

    @property
    def items(self):
        return self.k * self.k if self.context else self.k

    def lengths(self) -> np.ndarray:
        out = np.zeros((self.m, self.items), np.int32)
        for i in range(self.m):
            cb = self.arr[i]
            for j in range(cb.num_items):
                out[i, j] = cb.items[j].bit_length
        return out

    def estimate(self) -> np.ndarray:
        return np.array([lib().huffman_estimate_size(ctypes.byref(self.arr[i]),
                                                     _ptr(np.ascontiguousarray(self.counts[i])))
                         for i in range(self.m)])

    def file_bytes(self) -> bytes:
        """huffman_codebooks.bin content (huffman_encoder.c:398-409)."""
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "cb.bin").encode()
            f = _libc.fopen(path, b"wb")
            _libc.fwrite(ctypes.byref(ctypes.c_uint32(self.m)), 4, 1, ctypes.c_void_p(f))
            for i in range(self.m):
                lib().huffman_codebook_save(ctypes.byref(self.arr[i]), ctypes.c_void_p(f))
            _libc.fclose(ctypes.c_void_p(f))
            with open(path, "rb") as fh:
                return fh.read()

    @classmethod
    def load_file(cls, path: str) -> "Codebooks":
        with open(path, "rb") as fh:
            m = int(np.frombuffer(fh.read(4), np.uint32)[0])
        obj = cls._empty(m)
        f = _libc.fopen(path.encode(), b"rb")
        _libc.fseek(ctypes.c_void_p(f), ctypes.c_long(4), 0)
        for i in range(m):
            lib().huffman_codebook_load(ctypes.byref(obj.arr[i]), ctypes.c_void_p(f))
        _libc.fclose(ctypes.c_void_p(f))
        obj.k = obj.arr[0].alphabet_size
        obj.context = bool(obj.arr[0].is_context)
        obj.counts = None
        return obj

    def close(self):
        if getattr(self, "arr", None) is not None:
            for i in range(self.m):
                if self.arr[i].items:
                    lib().huffman_codebook_destroy(ctypes.byref(self.arr[i]))
            self.arr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Tables:
    """Device code tables (pqh_tables_t): encode entries + decode lookup tables."""

    def __init__(self, ctx: Context, m: int, k: int, context: bool):
        self.ctx, self.m, self.k, self.context = ctx, m, k, bool(context)
        self.ptr = ctypes.c_void_p()
        st = lib().pqh_tables_alloc(ctx.ptr, m, k, int(context), ctypes.byref(self.ptr))
        if st:
            raise PqhError(st, "pqh_tables_alloc: " + ctx.last_error())

    @classmethod
    def from_codebooks(cls, ctx: Context, cbs: "Codebooks") -> "Tables":
        t = cls(ctx, cbs.m, cbs.k, cbs.context)
        st = lib().pqh_tables_upload(ctx.ptr, t.ptr, ctypes.cast(cbs.arr, ctypes.c_void_p))
        if st:
            raise PqhError(st, "pqh_tables_upload: " + ctx.last_error())
        return t

    TREES = {None: 0, "lane": 1, "wave": 2, "grp": 3}

    def build(self, counts, ctx: Context = None, trees: str = None) -> "Tables":
        """GPU codebook construction from device counts (async, on `ctx`'s stream: any
        context of the same device, default the one the tables were allocated with).
        trees: the tree builder (pqh_tables_build_impl) -- None = the library default,
        "lane" (one lane per tree) or "wave" (one wavefront per tree); all build the same
        tables."""
        c = ctx or self.ctx
        check(lib().pqh_tables_build_impl(c.ptr, self.ptr, _ptr(counts), self.TREES[trees]),
              "pqh_tables_build")
        return self

    def build_trees(self, counts, ctx: Context = None, trees: str = None) -> "Tables":
        """The first half of build(): the Huffman trees only (on `ctx`'s stream)."""
        c = ctx or self.ctx
        check(lib().pqh_tables_build_trees(c.ptr, self.ptr, _ptr(counts), self.TREES[trees]),
              "pqh_tables_build_trees")
        return self

    def build_pair(self, counts, other: "Tables", counts2, ctx: Context = None) -> "Tables":
        """This table set from `counts` and `other` from `counts2` in one tree launch
        (pqh_tables_build_pair: the same tables as two build() calls)."""
        c = ctx or self.ctx
        check(lib().pqh_tables_build_pair(c.ptr, self.ptr, _ptr(counts), other.ptr, _ptr(counts2)),
              "pqh_tables_build_pair")
        return self

    def build_luts(self, ctx: Context = None) -> "Tables":
        """The second half of build(): decode tables + the encoder's gather copy, on
        `ctx`'s stream, which the caller has ordered behind build_trees (an event)."""
        c = ctx or self.ctx
        check(lib().pqh_tables_build_luts(c.ptr, self.ptr), "pqh_tables_build_luts")
        return self

    def encode_ready(self) -> bool:
        """whether the last build_trees completed the encoder's tables (the group builder
        writes the gather copy itself), so an encode need not wait for build_luts"""
        return bool(lib().pqh_tables_encode_ready(self.ptr))

    def status(self) -> None:
        st = lib().pqh_tables_status(self.ctx.ptr, self.ptr)
        if st:
            raise PqhError(st, "pqh_tables: " + self.ctx.last_error())

    def codebooks(self, counts_host=None) -> "Codebooks":
        cbs = Codebooks._empty(self.m)
        st = lib().pqh_tables_codebooks(self.ctx.ptr, self.ptr, ctypes.cast(cbs.arr, ctypes.c_void_p))
        if st:
            raise PqhError(st, "pqh_tables_codebooks: " + self.ctx.last_error())
        cbs.k, cbs.context, cbs.counts = self.k, self.context, counts_host
        return cbs

    def close(self):
        if self.ptr:
            lib().pqh_tables_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def histogram(ctx: Context, codes, k: int, context: bool, prev_row=None, counts=None,
              accumulate: bool = True):
    """counts (+)= the symbol histogram of codes (huffman_encoder.c:139-205);
    accumulate=False overwrites `counts` (pqh_histogram_set: no zeroing pass)."""
    torch = _torch()
    n, m = codes.shape
    items = k * k if context else k
    if counts is None:
        counts = torch.empty((m, items), dtype=torch.int32, device=codes.device)
        accumulate = False
    fn = lib().pqh_histogram if accumulate else lib().pqh_histogram_set
    check(fn(ctx.ptr, _ptr(codes), n, m, k, int(context), _ptr(prev_row), _ptr(counts)),
          "pqh_histogram")
    return counts


def histogram_partial_bytes(n: int, m: int, k: int) -> int:
    return int(lib().pqh_histogram_partial_bytes(n, m, k))


def histogram_partial(ctx: Context, codes, k: int, partials, prev_row=None):
    """First half of the context histogram: per-chunk partial pair counts into `partials`
    (a device byte buffer of histogram_partial_bytes(n, m, k)); pqh_histogram_partial."""
    n, m = codes.shape
    check(lib().pqh_histogram_partial(ctx.ptr, _ptr(codes), n, m, k, _ptr(prev_row),
                                      _ptr(partials)), "pqh_histogram_partial")
    return partials


def histogram_parts(ctx: Context, parts, n: int, k: int, context: bool, prev_row=None,
                    counts=None, accumulate: bool = True):
    """histogram() of part-major codes parts (m, >= n) (pqh_histogram_parts)."""
    torch = _torch()
    m = parts.shape[0]
    items = k * k if context else k
    if counts is None:
        counts = torch.empty((m, items), dtype=torch.int32, device=parts.device)
        accumulate = False
    check(lib().pqh_histogram_parts(ctx.ptr, _ptr(parts), parts.stride(0), n, m, k, int(context),
                                    _ptr(prev_row), _ptr(counts), 0 if accumulate else 1),
          "pqh_histogram_parts")
    return counts


def histogram_partial_parts(ctx: Context, parts, n: int, k: int, partials, prev_row=None):
    """histogram_partial() of part-major codes (pqh_histogram_partial_parts)."""
    m = parts.shape[0]
    check(lib().pqh_histogram_partial_parts(ctx.ptr, _ptr(parts), parts.stride(0), n, m, k,
                                            _ptr(prev_row), _ptr(partials)),
          "pqh_histogram_partial_parts")
    return partials


def transpose_codes(ctx: Context, parts, n: int, rows=None):
    """part-major codes (m, >= n) -> rows (n, m) (pqh_transpose_codes)."""
    torch = _torch()
    m = parts.shape[0]
    if rows is None:
        rows = torch.empty((n, m), dtype=parts.dtype, device=parts.device)
    check(lib().pqh_transpose_codes(ctx.ptr, _ptr(parts), parts.stride(0), n, m,
                                    parts.element_size(), _ptr(rows)), "pqh_transpose_codes")
    return rows


def histogram_reduce(ctx: Context, partials, n: int, m: int, k: int, counts,
                     accumulate: bool = False):
    """Second half: counts (+)= the sum of the partials (pqh_histogram_reduce)."""
    check(lib().pqh_histogram_reduce(ctx.ptr, _ptr(partials), n, m, k, _ptr(counts),
                                     0 if accumulate else 1), "pqh_histogram_reduce")
    return counts


def sort_rows(ctx: Context, codes, tmp=None):
    """In-place stable sort of uint8 code rows in strncmp order -- the reference encoder's
    default mode (huffman_encoder.c:301-317).  `tmp`: optional n*m byte device scratch."""
    n, m = codes.shape
    check(lib().pqh_sort_rows(ctx.ptr, _ptr(codes), n, m, _ptr(tmp)), "pqh_sort_rows")
    return codes


def counts_to_host(counts) -> np.ndarray:
    """uint32 device counts -> float64 host counts (the reference keeps counts in double)."""
    return counts.cpu().numpy().view(np.uint32).astype(np.float64)


@dataclass
class Encoded:
    stream: object            # device uint8, length padded to a multiple of 4
    bits: int
    chunk_vectors: int
    chunk_offsets: object     # device int64 [chunks]
    chunk_prev: object        # device codes [chunks, m] (context) or None
    n: int
    raw_first: int

    @property
    def nbytes(self) -> int:
        return (self.bits + 7) // 8


def encode_size(ctx: Context, tables: Tables, codes, raw_first: int = 1, prev_row=None):
    """device int64[1] total bits (async)."""
    torch = _torch()
    total = torch.zeros(1, dtype=torch.int64, device=codes.device)
    check(lib().pqh_encode_size(ctx.ptr, tables.ptr, _ptr(codes), codes.shape[0], raw_first,
                                _ptr(prev_row), _ptr(total)), "pqh_encode_size")
    return total


def encode_write(ctx: Context, tables: Tables, codes, out, bit_offset: int = 0, raw_first: int = 1,
                 prev_row=None, chunk_vectors: int = 64, chunk_offsets=None, chunk_prev=None,
                 total=None):
    """One-pass encode into `out` at `bit_offset` (no zeroing needed; bits of the first word
    before bit_offset are kept).  total: optional device int64[1] receiving the bit count."""
    check(lib().pqh_encode_write(ctx.ptr, tables.ptr, _ptr(codes), codes.shape[0], raw_first,
                                 _ptr(prev_row), bit_offset, _ptr(out), out.numel(),
                                 chunk_vectors, _ptr(chunk_offsets), _ptr(chunk_prev),
                                 _ptr(total)),
          "pqh_encode_write: " + ctx.last_error())
    return total


def encode_write_parts(ctx: Context, tables: Tables, parts, n: int, out, bit_offset: int = 0,
                       raw_first: int = 1, prev_row=None, chunk_vectors: int = 64,
                       chunk_offsets=None, chunk_prev=None, total=None):
    """encode_write() of part-major codes parts (m, >= n) (pqh_encode_write_parts)."""
    check(lib().pqh_encode_write_parts(ctx.ptr, tables.ptr, _ptr(parts), parts.stride(0), n,
                                       raw_first, _ptr(prev_row), bit_offset, _ptr(out),
                                       out.numel(), chunk_vectors, _ptr(chunk_offsets),
                                       _ptr(chunk_prev), _ptr(total)),
          "pqh_encode_write_parts: " + ctx.last_error())
    return total


def encode_write_at(ctx: Context, tables: Tables, codes, out, global_bit_offset, raw_first: int = 1,
                    prev_row=None, chunk_vectors: int = 64, chunk_offsets=None, chunk_prev=None,
                    total=None):
    """encode_write for one shard of a multi-GPU stream: the shard's global bit offset is a
    device int64[1] (shard.bit_offsets_device), so no host round trip; the shard lands at
    bit (offset % 32) of `out`."""
    check(lib().pqh_encode_write_at(ctx.ptr, tables.ptr, _ptr(codes), codes.shape[0], raw_first,
                                    _ptr(prev_row), _ptr(global_bit_offset), _ptr(out),
                                    out.numel(), chunk_vectors, _ptr(chunk_offsets),
                                    _ptr(chunk_prev), _ptr(total)),
          "pqh_encode_write_at: " + ctx.last_error())
    return total


def encode(ctx: Context, tables: Tables, codes, chunk_vectors: int = 64, raw_first: int = 1,
           prev_row=None) -> Encoded:
    torch = _torch()
    n, m = codes.shape
    total = encode_size(ctx, tables, codes, raw_first, prev_row)
    bits = int(total.item())
    words = (bits + 31) // 32 + 1
    out = torch.zeros(words * 4, dtype=torch.uint8, device=codes.device)
    chunks = (n + chunk_vectors - 1) // chunk_vectors
    coff = torch.empty(max(chunks, 1), dtype=torch.int64, device=codes.device)
    cprev = torch.empty((max(chunks, 1), m), dtype=codes.dtype, device=codes.device) \
        if tables.context else None
    encode_write(ctx, tables, codes, out, 0, raw_first, prev_row, chunk_vectors, coff, cprev)
    encode_status(ctx)
    return Encoded(out, bits, chunk_vectors, coff, cprev, n, raw_first)


def decode(ctx: Context, tables: Tables, enc: Encoded, out=None):
    torch = _torch()
    dt = torch.uint8 if tables.k <= 256 else torch.int16
    if out is None:
        out = torch.empty((enc.n, tables.m), dtype=dt, device=enc.stream.device)
    check(lib().pqh_decode(ctx.ptr, tables.ptr, _ptr(enc.stream), enc.stream.numel(), enc.n,
                           enc.raw_first, enc.chunk_vectors, _ptr(enc.chunk_offsets),
                           _ptr(enc.chunk_prev), _ptr(out)), "pqh_decode")
    return out


def encode_status(ctx: Context) -> None:
    st = lib().pqh_encode_status(ctx.ptr)
    if st:
        raise PqhError(st, "pqh_encode_write")


def decode_status(ctx: Context) -> None:
    st = lib().pqh_decode_status(ctx.ptr)
    if st:
        raise PqhError(st, "pqh_decode")


def indices_file_bytes(enc: Encoded) -> bytes:
    """huffman_indices.bin content: u64 N + stream bytes."""
    body = enc.stream[:enc.nbytes].cpu().numpy().tobytes()
    return np.uint64(enc.n).tobytes() + body


# ---- tree-ordered context coding (huffman_encoder.c --tree; mst.c:253-490) ---------------
def load_tree(path: str):
    """mst.tree (tree_save_file, mst.c:253-265): i64 N, i64 E, u32 targets[E], i32 counts[N].
    Returns (n, targets, counts)."""
    with open(path, "rb") as fh:
        raw = fh.read()
    n, e = (int(v) for v in np.frombuffer(raw[:16], np.int64))
    if len(raw) < 16 + 4 * e + 4 * n:
        raise ValueError(f"{path}: truncated tree file")
    targets = np.frombuffer(raw[16:16 + 4 * e], np.uint32).copy()
    counts = np.frombuffer(raw[16 + 4 * e:16 + 4 * e + 4 * n], np.int32).copy()
    return n, targets, counts


def tree_order(targets, counts):
    """DFS order of the forest (tree_collect_vertices_dfs, mst.c:290-364) and each stream
    row's coding context (tree_traverser, mst.c:366-405), by the library's host walk.
    Returns (vertices u32[n], num_children i32[n], parents i64[n] (-1: root), num_roots)."""
    targets = np.ascontiguousarray(targets, np.uint32)
    counts = np.ascontiguousarray(counts, np.int32)
    n = len(counts)
    vert = np.zeros(max(n, 1), np.uint32)
    nch = np.zeros(max(n, 1), np.int32)
    par = np.zeros(max(n, 1), np.int64)
    roots = lib().pqh_tree_order(n, len(targets), _ptr(targets), _ptr(counts), _ptr(vert),
                                 _ptr(nch), _ptr(par))
    if roots < 0:
        raise PqhError(roots, "pqh_tree_order: malformed forest")
    return vert[:n], nch[:n], par[:n], roots


def tree_order_device(ctx: Context, targets, counts):
    """tree_order on the device (pqh_tree_order_device): targets / counts as host arrays or
    device tensors.  Returns (vertices i32, num_children i32, parents i64) device tensors and
    num_roots, or None when the graph is not a forest (tree_order walks any graph)."""
    torch = _torch()
    dev = torch.device("cuda", ctx.device)
    t = torch.as_tensor(np.asarray(targets, np.uint32).view(np.int32)
                        if not torch.is_tensor(targets) else targets).to(dev, torch.int32)
    c = torch.as_tensor(np.asarray(counts, np.int32) if not torch.is_tensor(counts)
                        else counts).to(dev, torch.int32)
    n = c.numel()
    vert = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    nch = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    par = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    roots = ctypes.c_int(0)
    rc = lib().pqh_tree_order_device(ctx.ptr, n, t.numel(), _ptr(t), _ptr(c), _ptr(vert),
                                     _ptr(nch), _ptr(par), ctypes.byref(roots))
    if rc == -4:   # PQH_ERR_UNSUPPORTED
        return None
    check(rc, "pqh_tree_order_device: " + ctx.last_error())
    return vert[:n], nch[:n], par[:n], roots.value


@dataclass
class TreeEncoded:
    stream: object             # device uint8 (huffman_indices.bin payload), padded to 4 B
    bits: int
    n: int
    num_roots: int
    tables: object             # Tables (context, m parts)
    vertices: np.ndarray       # stream row p is input row vertices[p]
    num_children: np.ndarray
    children_codebook: object  # Codebooks (one non-context book, alphabet max + 1)
    children: object           # Encoded: the children stream (huffman_children.bin)
    chunk_vectors: int = 0     # decode sidecar: chunk bit offsets (device int64 [chunks])
    chunk_offsets: object = None
    ext_rows: object = None    # device uint8 [ext, m]: contexts that precede their chunk

    @property
    def nbytes(self) -> int:
        return (self.bits + 7) // 8


def tree_ext_index(num_children, chunk_vectors: int):
    """(parent_pos i64[n], ext_offsets i64[chunks + 1], ext_positions i64[ext]) -- the
    decode-side index of a tree stream (pqh_tree_ext_index)."""
    nch = np.ascontiguousarray(num_children, np.int32)
    n = len(nch)
    chunks = (n + chunk_vectors - 1) // chunk_vectors
    pp = np.zeros(max(n, 1), np.int64)
    eo = np.zeros(chunks + 1, np.int64)
    cnt = lib().pqh_tree_ext_index(n, _ptr(nch), chunk_vectors, _ptr(pp), _ptr(eo), None)
    if cnt < 0:
        raise PqhError(int(cnt), "pqh_tree_ext_index")
    ep = np.zeros(max(cnt, 1), np.int64)
    lib().pqh_tree_ext_index(n, _ptr(nch), chunk_vectors, _ptr(pp), _ptr(eo), _ptr(ep))
    return pp[:n], eo, ep[:cnt]


def tree_encode(ctx: Context, codes, targets, counts, chunk_vectors: int = 16) -> TreeEncoded:
    """Tree mode of huffman_encoder (huffman_encoder.c:321-375, encode_tree_data :240-286)
    on device uint8 codes [n, m]: DFS order (device Euler tour; the host walk for a graph
    that is not a forest) -> device gather of the rows in stream order
    beside their parents' codes -> parent/child pair histogram -> GPU code tables -> one-pass
    encode with explicit contexts; plus the children-count stream (non-context code book of
    tree_collect_num_children_stats, mst.c:407-440, coded by the GPU encoder).
    chunk_vectors: rows per decode lane (16: ~4x the lanes of 64 at ~10 % more sidecar)."""
    torch = _torch()
    n, m = codes.shape
    if len(counts) != n:
        raise ValueError(f"tree has {len(counts)} vertices for {n} rows")
    dev = codes.device
    order = tree_order_device(ctx, targets, counts)
    if order is not None:
        d_vert, d_nch, d_par, roots = order
        vert, nch = d_vert.cpu().numpy().view(np.uint32), d_nch.cpu().numpy()
    else:   # not a forest: the host walk reproduces the reference's DFS on any graph
        vert, nch, par, roots = tree_order(targets, counts)
        d_vert = torch.from_numpy(vert.astype(np.int32)).to(dev)
        d_par = torch.from_numpy(par).to(dev)
        d_nch = torch.from_numpy(np.ascontiguousarray(nch, np.int32)).to(dev)
    rows = torch.empty((n, m), dtype=torch.uint8, device=dev)
    prev = torch.empty((n, m), dtype=torch.int16, device=dev)
    check(lib().pqh_tree_gather(ctx.ptr, _ptr(codes), n, m, 256, _ptr(d_vert), _ptr(d_par),
                                _ptr(rows), _ptr(prev)), "pqh_tree_gather")
    check(lib().pqh_tree_status(ctx.ptr), "pqh_tree_gather: " + ctx.last_error())
    cnt = torch.zeros((m, 256 * 256), dtype=torch.int32, device=dev)
    check(lib().pqh_histogram_tree(ctx.ptr, _ptr(rows), _ptr(prev), n, m, 256, _ptr(cnt)),
          "pqh_histogram_tree")
    tables = Tables(ctx, m, 256, True).build(cnt)
    tables.status()
    words = (n * m * 56 + 31) // 32 + 2          # 56-bit codes at most
    out = torch.zeros(words * 4, dtype=torch.uint8, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    chunks = (n + chunk_vectors - 1) // chunk_vectors
    coff = torch.empty(max(chunks, 1), dtype=torch.int64, device=dev)
    check(lib().pqh_encode_tree_write(ctx.ptr, tables.ptr, _ptr(rows), _ptr(prev), n, 0,
                                      _ptr(out), out.numel(), chunk_vectors, _ptr(coff),
                                      _ptr(total)),
          "pqh_encode_tree_write: " + ctx.last_error())
    # decode sidecar: the contexts each chunk needs from before it (the encoder has them)
    _, _, _, ext_pos = tree_ext_index_device(ctx, d_nch, chunk_vectors, positions=True)
    ext_rows = rows.index_select(0, ext_pos)
    encode_status(ctx)
    bits = int(total.item())
    # children stream: one non-context part over the child counts
    alphabet = int(nch.max(initial=0)) + 1
    if alphabet > 4096:
        raise PqhError(-4, f"tree_encode: {alphabet - 1} children at one vertex (max 4095)")
    ccounts = np.bincount(nch, minlength=alphabet).astype(np.float64)[None]
    cbook = Codebooks(ccounts, alphabet, False)
    ctab = Tables.from_codebooks(ctx, cbook)
    ccodes = d_nch.to(torch.uint8 if alphabet <= 256 else torch.int16).reshape(n, 1)
    children = encode(ctx, ctab, ccodes, chunk_vectors=64, raw_first=1)
    return TreeEncoded(out, bits, n, roots, tables, vert, nch, cbook, children, chunk_vectors,
                       coff, ext_rows)


def tree_ext_index_device(ctx: Context, num_children, chunk_vectors: int,
                          positions: bool = False):
    """tree_ext_index on the device (pqh_tree_ext_index_device) from a device tensor of child
    counts (uint8, int16-as-u16 or int32): (parent_pos i64[n], ext_offsets i64[chunks + 1])
    device tensors and the ext count -- plus ext_positions i64[ext] with positions=True."""
    torch = _torch()
    nch = num_children.contiguous()
    n = nch.numel()
    nbytes = {torch.uint8: 1, torch.int16: 2, torch.int32: 4}[nch.dtype]
    chunks = (n + chunk_vectors - 1) // chunk_vectors
    pp = torch.empty(max(n, 1), dtype=torch.int64, device=nch.device)
    eo = torch.empty(chunks + 1, dtype=torch.int64, device=nch.device)
    ep = torch.empty(max(n, 1), dtype=torch.int64, device=nch.device) if positions else None
    ext = lib().pqh_tree_ext_index_device(ctx.ptr, n, _ptr(nch), nbytes, chunk_vectors,
                                          _ptr(pp), _ptr(eo), _ptr(ep) if positions else None)
    if ext < 0:
        raise PqhError(int(ext), "pqh_tree_ext_index_device: " + ctx.last_error())
    if positions:
        return pp[:n], eo, int(ext), ep[:ext]
    return pp[:n], eo, int(ext)


def tree_decode(ctx: Context, enc: TreeEncoded, tables: Tables = None, out=None,
                stream_bytes: int = None):
    """huffman_decoder --tree on the GPU (huffman_decoder.c:214-247): the children stream
    first (GPU decode of its non-context book), then the traverser's index over the decoded
    child counts (on the device), then one lane per chunk with the encoder's sidecar.  Rows come back in
    stream (DFS) order, as the reference decoder writes them.  stream_bytes (default: the
    encoded length) bounds the bits the decoder may consume: a stream shorter than its
    sidecar says raises PqhError (PQH_ERR_CORRUPT)."""
    torch = _torch()
    t = tables or enc.tables
    ctab = Tables.from_codebooks(ctx, enc.children_codebook)
    nch = decode(ctx, ctab, enc.children)
    decode_status(ctx)
    # the traverser's index on the device, from the decoded child counts in place
    d_pp, d_eo, _ = tree_ext_index_device(ctx, nch.reshape(-1), enc.chunk_vectors)
    dev = enc.stream.device
    if out is None:
        out = torch.empty((enc.n, t.m), dtype=torch.uint8, device=dev)
    nb = enc.nbytes if stream_bytes is None else stream_bytes
    check(lib().pqh_decode_tree(ctx.ptr, t.ptr, _ptr(enc.stream), nb, enc.n,
                                enc.chunk_vectors, _ptr(enc.chunk_offsets), _ptr(d_pp),
                                _ptr(d_eo), _ptr(enc.ext_rows), _ptr(out)), "pqh_decode_tree")
    decode_status(ctx)
    return out


def tree_files(enc: TreeEncoded) -> dict:
    """The reference's tree-mode output files (huffman_encoder.c:343-375, :398-428)."""
    cb = enc.tables.codebooks()
    stream = enc.stream[:enc.nbytes].cpu().numpy().tobytes()
    cstream = enc.children.stream[:enc.children.nbytes].cpu().numpy().tobytes()
    return {"huffman_codebooks.bin": cb.file_bytes(),
            "huffman_indices.bin": np.uint64(enc.n).tobytes() + stream,
            "huffman_children_codebooks.bin": enc.children_codebook.file_bytes()[4:],
            "huffman_children.bin": cstream}
