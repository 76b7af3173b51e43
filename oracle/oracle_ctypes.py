"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
_LIB = os.path.join(_HERE, "_build", "liboracle.so")
_LIB_O0 = os.path.join(_HERE, "_build", "liboracle_O0.so")   # -O0 -g (the reference's build)
_lib = None
_libs = {}

P, I, LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong


def build() -> None:
    subprocess.check_call(["make", "-s", "-f", "oracle/Makefile"], cwd=_ROOT)


def lib():
    global _lib
    if _lib is None:
        _lib = _load(_LIB)
    return _lib


def use_build(opt: str) -> None:
    """Route this module's functions to the -O2 (default) or the -O0 -g build."""
    global _lib
    path = _LIB_O0 if opt == "O0" else _LIB
    if path not in _libs:
        _libs[path] = _load(path)
    _lib = _libs[path]


def _load(path):
    if True:
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.orc_codebook.argtypes = [I, I, P, P, P, I]
        L.orc_codebook.restype = I
        L.orc_codebook_serialize.argtypes = [I, I, P, P, I, P, LL]
        L.orc_codebook_serialize.restype = LL
        L.orc_histogram.argtypes = [P, I, LL, I, I, I, P]
        L.orc_encode.argtypes = [P, I, LL, I, I, I, P, P, I, P, LL]
        L.orc_encode.restype = LL
        L.orc_decode.argtypes = [P, LL, LL, I, I, I, P, P, I, P, I]
        L.orc_decode.restype = I
        L.orc_sort_rows.argtypes = [P, LL, I]
        L.orc_pq_assign.argtypes = [P, LL, I, I, I, P, P, I, P, I]
        L.orc_kmeans.argtypes = [P, LL, I, I, I, I, P, I]
        L.orc_kmeans_shift.argtypes = [ctypes.c_float, LL]
        L.orc_kmeans_shift.restype = I
        L.orc_compute_error.argtypes = [P, LL, I, I, I, P, P, I]
        L.orc_compute_error.restype = ctypes.c_double
        L.orc_estimate_size.argtypes = [P, P, LL]
        L.orc_estimate_size.restype = ctypes.c_double
        L.orc_stats_json.argtypes = [LL, I, I, I, P, ctypes.c_char_p, I]
        L.orc_stats_json.restype = I
        L.orc_bitstream_write.argtypes = [P, P, I, P, LL]
        L.orc_decode_tree.argtypes = [P, LL, LL, I, I, P, P, I, P, P]
        L.orc_tree_order.argtypes = [LL, LL, P, P, P, P]
        L.orc_tree_parents.argtypes = [LL, P, P, P]
        L.orc_tree_histogram.argtypes = [P, LL, I, I, P, P, P]
        L.orc_tree_encode.argtypes = [P, LL, I, I, P, P, P, P, I, P, LL]
        L.orc_tree_encode.restype = LL
        L.orc_bitstream_write.restype = LL
        L.orc_knn_blocks_info.argtypes = [P, LL, I, I, I, ctypes.c_double, P, P]
        L.orc_in_block.argtypes = [P, I, I, P, P, LL]
        L.orc_in_block.restype = I
        L.orc_knn_fast.argtypes = [P, LL, I, I, I, I, P, P, P, P, P, P, P, P, P]
        L.orc_mst.argtypes = [LL, I, I, P, P, I, ctypes.c_float, P, P, P]
        L.orc_mst.restype = LL
        _libs[path] = L
        return L


def bitstream_write(data: np.ndarray, lens: np.ndarray) -> bytes:
    data = np.ascontiguousarray(data, np.uint8)
    lens = np.ascontiguousarray(lens, np.int64)
    cap = int(lens.sum()) // 8 + 8
    out = np.zeros(cap, np.uint8)
    n = lib().orc_bitstream_write(_p(data), _p(lens), len(lens), _p(out), cap)
    assert n >= 0
    return out[:n].tobytes()


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Codebooks:
    """m codebooks: lens [m][items] int32, codes [m][items][stride] uint8."""

    def __init__(self, k: int, context: bool, lens, codes, stride: int):
        self.k, self.context, self.lens, self.codes, self.stride = k, context, lens, codes, stride

    @property
    def items(self):
        return self.k * self.k if self.context else self.k


def codebook(alphabet: int, counts: np.ndarray, context: bool = False, stride: int | None = None):
    rows = alphabet if context else 1
    stride = stride or max(8, (alphabet + 7) // 8 + 1)
    counts = np.ascontiguousarray(counts, np.float64)
    lens = np.zeros(rows * alphabet, np.int32)
    codes = np.zeros((rows * alphabet, stride), np.uint8)
    rc = lib().orc_codebook(alphabet, rows, _p(counts), _p(lens), _p(codes), stride)
    if rc < 0:
        raise ValueError("code longer than stride")
    return lens, codes


def serialize(alphabet: int, context: bool, lens, codes) -> bytes:
    items = alphabet * alphabet if context else alphabet
    cap = 5 + items * 4 + int(lens.sum()) // 8 + 16
    out = np.zeros(cap, np.uint8)
    n = lib().orc_codebook_serialize(alphabet, int(context), _p(lens), _p(codes),
                                     codes.shape[1], _p(out), cap)
    assert n >= 0
    return out[:n].tobytes()


def histogram(codes: np.ndarray, k: int, context: bool) -> np.ndarray:
    codes = np.ascontiguousarray(codes)
    n, m = codes.shape
    per = k * k if context else k
    out = np.zeros(m * per, np.float64)
    lib().orc_histogram(_p(codes), codes.itemsize, n, m, k, int(context), _p(out))
    return out.reshape(m, per)


def build_codebooks(codes: np.ndarray, k: int, context: bool, stride: int = 8) -> Codebooks:
    counts = histogram(codes, k, context)
    m = codes.shape[1]
    items = k * k if context else k
    lens = np.zeros((m, items), np.int32)
    cds = np.zeros((m, items, stride), np.uint8)
    for i in range(m):
        lens[i], cds[i] = codebook(k, counts[i], context, stride)
    return Codebooks(k, context, lens, cds, stride)


def codebooks_file(cbs: Codebooks) -> bytes:
    m = cbs.lens.shape[0]
    parts = [np.uint32(m).tobytes()]
    for i in range(m):
        parts.append(serialize(cbs.k, cbs.context, cbs.lens[i], cbs.codes[i]))
    return b"".join(parts)


def encode(codes: np.ndarray, cbs: Codebooks) -> tuple[bytes, int]:
    codes = np.ascontiguousarray(codes)
    n, m = codes.shape
    cap = int(cbs.lens.max(initial=8) + 8) * n * m // 8 + 64
    out = np.zeros(cap, np.uint8)
    bits = lib().orc_encode(_p(codes), codes.itemsize, n, m, cbs.k, int(cbs.context),
                            _p(cbs.lens), _p(cbs.codes), cbs.stride, _p(out), cap)
    assert bits >= 0
    return out[:(bits + 7) // 8].tobytes(), bits


def indices_file(codes: np.ndarray, cbs: Codebooks) -> bytes:
    stream, _ = encode(codes, cbs)
    return np.uint64(codes.shape[0]).tobytes() + stream


def decode(stream: bytes, n: int, m: int, cbs: Codebooks) -> np.ndarray:
    buf = np.frombuffer(stream, np.uint8).copy() if len(stream) else np.zeros(1, np.uint8)
    dt = np.uint8 if cbs.k <= 256 else np.uint16
    out = np.zeros((n, m), dt)
    rc = lib().orc_decode(_p(buf), len(stream), n, m, cbs.k, int(cbs.context), _p(cbs.lens),
                          _p(cbs.codes), cbs.stride, _p(out), out.itemsize)
    if rc != 0:
        raise ValueError(f"oracle decode failed rc={rc}")
    return out


def sort_rows(codes: np.ndarray) -> np.ndarray:
    out = np.ascontiguousarray(codes, np.uint8).copy()
    lib().orc_sort_rows(_p(out), out.shape[0], out.shape[1])
    return out


def kmeans(x: np.ndarray, init: np.ndarray, iters: int, threads: int = 0) -> np.ndarray:
    """Deterministic fixed-point Lloyd (the build's training definition); init [m][k][ds]."""
    x = np.ascontiguousarray(x, np.float32)
    cent = np.ascontiguousarray(init, np.float32).copy()
    m, k, ds = cent.shape
    lib().orc_kmeans(_p(x), x.shape[0], x.shape[1], m, k, iters, _p(cent), threads)
    return cent


def pq_assign(x: np.ndarray, centroids: np.ndarray, threads: int = 1):
    x = np.ascontiguousarray(x, np.float32)
    centroids = np.ascontiguousarray(centroids, np.float32)
    m, k, ds = centroids.shape
    n, d = x.shape
    codes = np.zeros((n, m), np.uint8 if k <= 256 else np.uint16)
    dists = np.zeros((n, m), np.float32)
    lib().orc_pq_assign(_p(x), n, d, m, k, _p(centroids), _p(codes), codes.itemsize,
                        _p(dists), threads)
    return codes, dists


def compute_error(x, centroids, codes) -> float:
    x = np.ascontiguousarray(x, np.float32)
    centroids = np.ascontiguousarray(centroids, np.float32)
    codes = np.ascontiguousarray(codes)
    m, k, _ = centroids.shape
    return lib().orc_compute_error(_p(x), x.shape[0], x.shape[1], m, k, _p(centroids),
                                   _p(codes), codes.itemsize)


def stats_json(n: int, m: int, k: int, num_roots: int, partial) -> str:
    partial = np.ascontiguousarray(partial, np.float64)
    buf = ctypes.create_string_buffer(8192 + 256 * m)
    lib().orc_stats_json(n, m, k, num_roots, _p(partial), buf, len(buf))
    return buf.value.decode()


def estimate_parts(cbs: Codebooks, counts: np.ndarray) -> np.ndarray:
    return np.array([lib().orc_estimate_size(_p(np.ascontiguousarray(cbs.lens[i])),
                                             _p(np.ascontiguousarray(counts[i])), cbs.items)
                     for i in range(cbs.lens.shape[0])])


# ---- tree mode (huffman_encoder.c --tree; mst.c:290-490) --------------------------------
def tree_order(n: int, targets: np.ndarray, counts: np.ndarray):
    """(vertices u32, num_children i32, num_roots) -- tree_collect_vertices_dfs."""
    targets = np.ascontiguousarray(targets, np.uint32)
    counts = np.ascontiguousarray(counts, np.int32)
    vert = np.zeros(max(n, 1), np.uint32)
    nch = np.zeros(max(n, 1), np.int32)
    roots = lib().orc_tree_order(n, len(targets), _p(targets), _p(counts), _p(vert), _p(nch))
    assert roots >= 0
    return vert[:n], nch[:n], roots


def tree_parents(num_children: np.ndarray, ids=None) -> np.ndarray:
    """Active traverser parent per stream row (ids=None: stream positions, the decoder's)."""
    nch = np.ascontiguousarray(num_children, np.int32)
    n = len(nch)
    out = np.zeros(max(n, 1), np.int64)
    idp = None if ids is None else np.ascontiguousarray(ids, np.uint32)
    lib().orc_tree_parents(n, None if idp is None else _p(idp), _p(nch), _p(out))
    return out[:n]


def tree_histogram(codes: np.ndarray, vertices, parents, k: int = 256) -> np.ndarray:
    codes = np.ascontiguousarray(codes, np.uint8)
    n, m = codes.shape
    out = np.zeros(m * k * k, np.float64)
    v = np.ascontiguousarray(vertices, np.uint32)
    par = np.ascontiguousarray(parents, np.int64)
    lib().orc_tree_histogram(_p(codes), n, m, k, _p(v), _p(par), _p(out))
    return out.reshape(m, k * k)


def tree_codebooks(codes: np.ndarray, vertices, parents, stride: int = 8) -> Codebooks:
    counts = tree_histogram(codes, vertices, parents)
    m = codes.shape[1]
    lens = np.zeros((m, 256 * 256), np.int32)
    cds = np.zeros((m, 256 * 256, stride), np.uint8)
    for i in range(m):
        lens[i], cds[i] = codebook(256, counts[i], True, stride)
    return Codebooks(256, True, lens, cds, stride)


def tree_encode(codes: np.ndarray, vertices, parents, cbs: Codebooks) -> tuple[bytes, int]:
    codes = np.ascontiguousarray(codes, np.uint8)
    n, m = codes.shape
    cap = int(cbs.lens.max(initial=8) + 8) * n * m // 8 + 64
    out = np.zeros(cap, np.uint8)
    v = np.ascontiguousarray(vertices, np.uint32)
    par = np.ascontiguousarray(parents, np.int64)
    bits = lib().orc_tree_encode(_p(codes), n, m, 256, _p(v), _p(par), _p(cbs.lens),
                                 _p(cbs.codes), cbs.stride, _p(out), cap)
    assert bits >= 0
    return out[:(bits + 7) // 8].tobytes(), bits


def tree_decode(stream: bytes, n: int, m: int, cbs: Codebooks, num_children) -> np.ndarray:
    """Rows in stream (DFS) order, contexts from the children counts."""
    pos = tree_parents(num_children)
    buf = np.frombuffer(stream, np.uint8).copy() if len(stream) else np.zeros(1, np.uint8)
    out = np.zeros((n, m), np.uint8)
    rc = lib().orc_decode_tree(_p(buf), len(stream), n, m, 256, _p(cbs.lens), _p(cbs.codes),
                               cbs.stride, _p(out), _p(pos))
    if rc != 0:
        raise ValueError(f"oracle tree decode failed rc={rc}")
    return out


def children_codebook(num_children) -> tuple[np.ndarray, Codebooks]:
    """tree_collect_num_children_stats (mst.c:407-440) + its non-context codebook."""
    nch = np.asarray(num_children, np.int64)
    alphabet = int(nch.max(initial=0)) + 1
    counts = np.bincount(nch, minlength=alphabet).astype(np.float64)
    lens, cds = codebook(alphabet, counts, False)
    return counts, Codebooks(alphabet, False, lens[None], cds[None], cds.shape[1])


# ---- forest builder (compute_nn_fast.c, mst.c) ------------------------------------------
def knn_blocks_info(x: np.ndarray, num_split: int, blocks_per_dim: int, overlap: float):
    """(starts, ends) float32 [num_split][blocks_per_dim] -- blocks_info_init."""
    x = np.ascontiguousarray(x, np.float32)
    n, d = x.shape
    st = np.zeros((num_split, blocks_per_dim), np.float32)
    en = np.zeros_like(st)
    lib().orc_knn_blocks_info(_p(x), n, d, num_split, blocks_per_dim, overlap, _p(st), _p(en))
    return st, en


def knn_members(x: np.ndarray, starts, ends) -> list:
    """Rows of every block in block-id order (is_vector_in_block)."""
    x = np.ascontiguousarray(x, np.float32)
    st = np.ascontiguousarray(starts, np.float32)
    en = np.ascontiguousarray(ends, np.float32)
    ns, nb = st.shape
    L = lib()
    out = []
    for b in range(nb ** ns):
        out.append(np.array([v for v in range(x.shape[0])
                             if L.orc_in_block(_p(x[v]), ns, nb, _p(st), _p(en), b)], np.int64))
    return out


def knn_fast(x: np.ndarray, num_nn: int, starts, ends, log: bool = False):
    """(indices u32 [n][num_nn], dists f32, block_sizes[, (rows, idx, dist) push log])."""
    x = np.ascontiguousarray(x, np.float32)
    n, d = x.shape
    st = np.ascontiguousarray(starts, np.float32)
    en = np.ascontiguousarray(ends, np.float32)
    ns, nb = st.shape
    idx = np.zeros((max(n, 1), num_nn), np.uint32)
    dist = np.zeros((max(n, 1), num_nn), np.float32)
    sizes = np.zeros(nb ** ns, np.int64)
    if log:
        cap = n * num_nn * (nb ** ns) + 1
        lr, li, ld = np.zeros(cap, np.int64), np.zeros(cap, np.uint32), np.zeros(cap, np.float32)
        cnt = np.zeros(1, np.int64)
        lib().orc_knn_fast(_p(x), n, d, num_nn, ns, nb, _p(st), _p(en), _p(idx), _p(dist),
                           _p(sizes), _p(lr), _p(li), _p(ld), _p(cnt))
        c = int(cnt[0])
        return idx[:n], dist[:n], sizes, (lr[:c], li[:c], ld[:c])
    lib().orc_knn_fast(_p(x), n, d, num_nn, ns, nb, _p(st), _p(en), _p(idx), _p(dist),
                       _p(sizes), None, None, None, None)
    return idx[:n], dist[:n], sizes


def mst(indices: np.ndarray, dists: np.ndarray, take: int, pq=None, penalty: float = 0.0):
    """(targets u32 [num_edges], counts i32 [n]) -- the arrays of mst.tree."""
    idx = np.ascontiguousarray(indices, np.uint32)
    dist = np.ascontiguousarray(dists, np.float32)
    n, num_nn = idx.shape
    pqa = None if pq is None else np.ascontiguousarray(pq, np.uint8)
    pq_m = 0 if pqa is None else pqa.shape[1]
    targets = np.zeros(max(2 * n, 1), np.uint32)
    counts = np.zeros(max(n, 1), np.int32)
    ne = lib().orc_mst(n, num_nn, take, _p(idx), _p(dist), pq_m, penalty,
                       None if pqa is None else _p(pqa), _p(targets), _p(counts))
    assert ne >= 0, "neighbour id outside the rows"
    return targets[:ne], counts[:n]


def tree_file(n: int, targets: np.ndarray, counts: np.ndarray) -> bytes:
    """tree_save_file (mst.c:253-265): i64 N, i64 E, u32 targets[E], i32 counts[N]."""
    return (np.array([n, len(targets)], np.int64).tobytes() +
            np.ascontiguousarray(targets, np.uint32).tobytes() +
            np.ascontiguousarray(counts, np.int32).tobytes())
