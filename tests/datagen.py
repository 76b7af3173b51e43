"""Seeded synthetic inputs shared by tests/ and oracle/gen_golden.py (test infrastructure).

* ``skewed_codes`` -- PQ-code matrices shaped like real PQ output: geometric(p) symbols
  clipped to the alphabet (the generator BASELINE.md section 2 used for the reference
  timings), plus an order-1 correlation between consecutive vectors so that context
  coding has something to exploit.
* ``sift_like`` -- "SIFT-like" fp32 vectors: integer-valued, non-negative, in [0, 255],
  drawn from a Gaussian mixture with Zipf(1.1) cluster weights.
* ``deep_like`` -- unit-normalised mixture for the Deep-style config (C4).
"""
from __future__ import annotations

import numpy as np


def skewed_codes(n: int, m: int, k: int = 256, seed: int = 1, p: float = 0.02,
                 stay: float = 0.3) -> np.ndarray:
    rng = np.random.default_rng(seed)
    dtype = np.uint8 if k <= 256 else np.uint16
    base = np.minimum(rng.geometric(p, size=(n, m)) - 1, k - 1)
    # per-part permutation so parts have different popular symbols
    for j in range(m):
        base[:, j] = rng.permutation(k)[base[:, j]]
    if n > 1 and stay > 0:
        keep = rng.random((n, m)) < stay
        for v in range(1, n):
            row = keep[v]
            base[v, row] = base[v - 1, row]
    return base.astype(dtype)


def sift_like(n: int, d: int = 128, seed: int = 0x5EED, centers: int = 1024) -> np.ndarray:
    rng = np.random.default_rng(seed)
    mu = rng.gamma(1.2, 30.0, size=(centers, d)).astype(np.float32)
    w = 1.0 / np.arange(1, centers + 1) ** 1.1
    w /= w.sum()
    lab = rng.choice(centers, size=n, p=w)
    x = mu[lab] + rng.normal(0.0, 12.0, size=(n, d)).astype(np.float32)
    return np.clip(np.rint(x), 0, 255).astype(np.float32)


def deep_like(n: int, d: int = 96, seed: int = 0xDEE9, centers: int = 512) -> np.ndarray:
    rng = np.random.default_rng(seed)
    mu = rng.normal(0.0, 1.0, size=(centers, d)).astype(np.float32)
    lab = rng.integers(0, centers, size=n)
    x = mu[lab] + rng.normal(0.0, 0.35, size=(n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(np.float32)


def lloyd_centroids(x: np.ndarray, m: int, k: int, iters: int = 4, seed: int = 7,
                    sample: int = 20000) -> np.ndarray:
    """Deterministic per-subspace Lloyd k-means on a sample (test setup only).
    Returns centroids [m][k][d/m] in pq_centroids.fvecsl order."""
    rng = np.random.default_rng(seed)
    n, d = x.shape
    ds = d // m
    xs = x[rng.choice(n, size=min(sample, n), replace=False)]
    out = np.empty((m, k, ds), np.float32)
    for j in range(m):
        sub = xs[:, j * ds:(j + 1) * ds].astype(np.float64)
        c = sub[rng.choice(len(sub), size=k, replace=len(sub) < k)].copy()
        for _ in range(iters):
            dd = (sub ** 2).sum(1)[:, None] - 2 * sub @ c.T + (c ** 2).sum(1)[None]
            a = dd.argmin(1)
            sums = np.zeros_like(c)
            np.add.at(sums, a, sub)
            cnt = np.bincount(a, minlength=k)
            nz = cnt > 0
            c[nz] = sums[nz] / cnt[nz, None]
        out[j] = c.astype(np.float32)
    return out


def write_fvecs(path, x: np.ndarray) -> None:
    """.fvecs: per row int32 D then D float32 (pq_encoder.c:46-80)."""
    n, d = x.shape
    rows = np.empty((n, d + 1), np.float32)
    rows[:, 1:] = x
    rows.view(np.int32)[:, 0] = d
    rows.tofile(path)


def write_vecsl(path, a: np.ndarray) -> None:
    """light .xvecsl: u32 N, u32 D, raw payload (vecs_io.c:70-76)."""
    n, d = a.shape
    with open(path, "wb") as f:
        np.array([n, d], np.uint32).tofile(f)
        np.ascontiguousarray(a).tofile(f)


def random_forest(n: int, roots: int = 3, seed: int = 9, max_fan: int = 6):
    """A spanning forest of n vertices in the reference's mst.tree layout (mst.c:173-236):
    every edge stored in both directions, grouped by source vertex (order within a source
    arbitrary).  Returns (targets u32 [2(n - roots)], counts i32 [n])."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n)
    adj = [[] for _ in range(n)]
    roots = max(1, min(roots, n)) if n else 0
    for j in range(roots, n):          # attach perm[j] below a recent earlier vertex
        lo = max(0, j - max_fan * 4)
        par = perm[int(rng.integers(lo, j))] if j > lo else perm[0]
        adj[par].append(perm[j])
        adj[perm[j]].append(par)
    for a in adj:
        rng.shuffle(a)
    counts = np.array([len(a) for a in adj], np.int32)
    targets = np.array([t for a in adj for t in a], np.uint32)
    return targets, counts


def write_tree(path, n: int, targets: np.ndarray, counts: np.ndarray) -> None:
    """tree_save_file (mst.c:253-265): i64 N, i64 E, u32 targets[E], i32 counts[N]."""
    with open(path, "wb") as f:
        f.write(np.int64(n).tobytes())
        f.write(np.int64(len(targets)).tobytes())
        f.write(np.ascontiguousarray(targets, np.uint32).tobytes())
        f.write(np.ascontiguousarray(counts, np.int32).tobytes())


def read_tree(path):
    """tree_load_file (mst.c:273-288) -> (n, targets, counts)."""
    raw = open(path, "rb").read()
    n, e = np.frombuffer(raw[:16], np.int64)
    targets = np.frombuffer(raw[16:16 + 4 * e], np.uint32).copy()
    counts = np.frombuffer(raw[16 + 4 * e:16 + 4 * e + 4 * n], np.int32).copy()
    return int(n), targets, counts
