"""The forest builder of tree mode on the GPU: compute_nn_fast's blocked kNN graph and
mst_builder's minimum spanning forest (include/pqh.h "forest builder").

    starts, ends = blocks_info(ctx, x, num_split, blocks_per_dim, overlap)  # blocks_info_init
    idx, dist, sizes = knn_fast(ctx, x, num_nn, starts, ends)               # compute_nn_fast
    targets, counts = mst(ctx, idx, dist, take, pq_codes, penalty)          # mst_builder

x is a (n, d) float32 CUDA tensor (rows may be strided); the kNN lists stay on the device
((n, num_nn) uint32 / float32, as nn_indices.ivecsl / nn_dist.fvecsl hold them); the
forest comes back as the host arrays of mst.tree (tree_save_file, mst.c:253-265).  The
default geometry is the reference CLI's (compute_nn_fast.c:168-170: 5 splits, 3 blocks per
split, overlap 0.3); run.sh's nn-fast action uses 3 / 10 / 0.01.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .capi import check, lib
from .codec import Context, _torch


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _a(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _rows(x):
    if x.dim() != 2 or x.dtype != _torch().float32 or not x.is_cuda or x.stride(1) != 1:
        raise ValueError("x must be a (n, d) float32 CUDA tensor with unit column stride")
    return x.shape[0], x.shape[1], x.stride(0)


def blocks_info(ctx: Context, x, num_split: int = 5, blocks_per_dim: int = 3,
                overlap: float = 0.3):
    """(starts, ends) float32 [num_split][blocks_per_dim]: blocks_info_init
    (fast_nn_blocks_info.c:94-112) -- split i is coordinate num_split-1-i."""
    n, d, ld = _rows(x)
    st = np.zeros((num_split, blocks_per_dim), np.float32)
    en = np.zeros_like(st)
    check(lib().pqh_knn_blocks_info(ctx.ptr, _p(x), n, ld, d, num_split, blocks_per_dim,
                                    float(overlap), _a(st), _a(en)), "pqh_knn_blocks_info")
    return st, en


def knn_fast(ctx: Context, x, num_nn: int, starts, ends, indices=None, dists=None):
    """compute_nn_fast (one block per pass): (indices (n, num_nn) uint32 as int32 tensor,
    dists (n, num_nn) float32, block sizes) -- ascending per row, never-filled slots
    0xFFFFFFFF / +inf."""
    torch = _torch()
    n, d, ld = _rows(x)
    st = np.ascontiguousarray(starts, np.float32)
    en = np.ascontiguousarray(ends, np.float32)
    ns, nb = st.shape
    if indices is None:
        indices = torch.empty((n, num_nn), dtype=torch.int32, device=x.device)
    if dists is None:
        dists = torch.empty((n, num_nn), dtype=torch.float32, device=x.device)
    sizes = np.zeros(nb ** ns, np.int64)
    check(lib().pqh_knn_fast(ctx.ptr, _p(x), n, ld, d, num_nn, ns, nb, _a(st), _a(en),
                             _p(indices), _p(dists), _a(sizes)), "pqh_knn_fast")
    return indices, dists, sizes


def mst(ctx: Context, indices, dists, take: int, pq_codes=None, penalty: float = 0.0):
    """mst_builder's forest: (targets uint32 [num_edges], counts int32 [n]) of mst.tree."""
    n, num_nn = indices.shape
    targets = np.zeros(max(2 * n, 1), np.uint32)
    counts = np.zeros(max(n, 1), np.int32)
    ne = ctypes.c_longlong(0)
    pq_m = 0 if pq_codes is None else pq_codes.shape[1]
    check(lib().pqh_mst_build(ctx.ptr, _p(indices), _p(dists), n, num_nn, take,
                              None if pq_codes is None else _p(pq_codes), pq_m,
                              float(penalty), _a(targets), _a(counts), ctypes.byref(ne)),
          "pqh_mst_build")
    return targets[:ne.value], counts[:n]


def tree_file(n: int, targets: np.ndarray, counts: np.ndarray) -> bytes:
    """mst.tree bytes (tree_save_file, mst.c:253-265): i64 N, i64 E, u32 targets[E],
    i32 children_counts[N]."""
    return (np.array([n, len(targets)], np.int64).tobytes() +
            np.ascontiguousarray(targets, np.uint32).tobytes() +
            np.ascontiguousarray(counts, np.int32).tobytes())
