"""GPU parity of PQ assignment (pqh_pq_assign through the C ABI) against the CPU oracle:
bit-exact codes, first-minimum ties, non-finite inputs, both kernels."""
import numpy as np
import pytest

from conftest import golden
import datagen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    assert torch.cuda.is_available()
    ctx = codec.Context(0)
    return torch, codec, ctx


def _assign(gpu, x, cent, mode=0, counts=None):
    torch, codec, ctx = gpu
    pq = codec.PQ(ctx, cent)
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    codes = pq.assign(xd, counts=counts, mode=mode)
    out = codes.cpu().numpy()
    return out, pq.rerank_count()


@pytest.mark.parametrize("name", ["sift_n1000_m8_k256", "deep_n500_m16_k256"])
@pytest.mark.parametrize("mode", [0, 1])
def test_assign_golden(gpu, name, mode):
    g = golden(f"pq_{name}.npz")
    codes, _ = _assign(gpu, g["x"], g["centroids"], mode)
    assert np.array_equal(codes, g["codes"])


@pytest.mark.parametrize("kind,d,m", [("sift", 128, 8), ("deep", 96, 16), ("deep", 96, 8),
                                      ("sift", 128, 16), ("sift", 128, 32), ("sift", 64, 4),
                                      ("sift", 128, 4), ("deep", 96, 3)])
def test_assign_vs_oracle_random(gpu, oracle, kind, d, m):
    """Every dsub the MFMA kernel serves (4, 6, 8, 12, 16, 32): codes == oracle; the
    screening ran (near ties were re-ranked: the exact-only kernel reports none)."""
    n = 6001  # not a multiple of 32
    x = datagen.sift_like(n, d, seed=11) if kind == "sift" else datagen.deep_like(n, d, seed=12)
    cent = datagen.lloyd_centroids(x, m, 256, iters=2, sample=4000, seed=3)
    want, _ = oracle.pq_assign(x, cent, threads=0)
    got, rr = _assign(gpu, x, cent, 0)
    assert np.array_equal(got, want), (got != want).sum()
    assert rr > 0
    got1, _ = _assign(gpu, x, cent, 1)
    assert np.array_equal(got1, want)


def test_assign_ties_first_index(gpu, oracle):
    """Duplicate centroids: the first of equal distances must win (strict <)."""
    rng = np.random.default_rng(5)
    x = rng.integers(0, 50, (512, 32)).astype(np.float32)
    cent = rng.integers(0, 50, (2, 256, 16)).astype(np.float32)
    cent[:, 128:] = cent[:, :128]            # every centroid duplicated
    cent[0, 7] = x[3, :16]                    # exact hit (distance 0) ...
    cent[0, 200] = x[3, :16]                  # ... twice
    want, _ = oracle.pq_assign(x, cent)
    got, rr = _assign(gpu, x, cent)
    assert np.array_equal(got, want)
    assert got[3, 0] == 7
    assert rr > 0                             # ties must have gone to the exact re-rank


def test_assign_rerank_queue_overflow(gpu, oracle):
    """Every vector ties (duplicated centroids), so each wave's deferred re-rank segment
    (1024 entries) overflows and the rest is re-ranked inline; codes and the fused
    histogram must still match the oracle."""
    torch, codec, ctx = gpu
    rng = np.random.default_rng(17)
    n = 300_000
    x = rng.integers(0, 40, (n, 32)).astype(np.float32)
    cent = rng.integers(0, 40, (2, 256, 16)).astype(np.float32)
    cent[:, 128:] = cent[:, :128]
    want, _ = oracle.pq_assign(x, cent, threads=0)
    counts = torch.zeros((2, 256), dtype=torch.int32, device="cuda")
    got, rr = _assign(gpu, x, cent, 0, counts)
    assert np.array_equal(got, want), (got != want).sum()
    assert rr >= n                            # every vector re-ranked at least in one part
    assert np.array_equal(codec.counts_to_host(counts), oracle.histogram(got, 256, False))


@pytest.mark.parametrize("lo", [False, True])
def test_assign_one_tile_winners(gpu, oracle, lo):
    """Skewed data: every vector sits next to a centroid of tile 0 (rows 0-31), so every
    winner comes from one MFMA tile and one P-group pair; with `lo` the x are not bf16-exact
    (the lo MFMA pass).  Codes and fused counts == the oracle."""
    torch, codec, ctx = gpu
    rng = np.random.default_rng(23)
    n, m, dsub = 200_003, 4, 16
    cent = (rng.random((m, 256, dsub)) * 100).astype(np.float32)
    pick = rng.integers(0, 32, (n, m))
    x = np.empty((n, m * dsub), np.float32)
    for i in range(m):
        x[:, i * dsub:(i + 1) * dsub] = cent[i][pick[:, i]] + rng.normal(0, 0.5, (n, dsub))
    if not lo:
        x = np.round(x)
    x = x.astype(np.float32)
    want, _ = oracle.pq_assign(x, cent, threads=0)
    assert (want < 32).all()
    counts = torch.zeros((m, 256), dtype=torch.int32, device="cuda")
    got, _ = _assign(gpu, x, cent, 0, counts)
    assert np.array_equal(got, want), (got != want).sum()
    assert np.array_equal(codec.counts_to_host(counts), oracle.histogram(got, 256, False))


def test_assign_alternating_subspace_counts_one_context(gpu, oracle):
    """m = 16, then 8, then 16 on one context, each with enough rows for the dynamic work
    queues: a launch resets the next launch's queue heads (and spill counters) for every
    subspace, not only its own, so the third launch finds subspaces 8-15 fresh."""
    x = datagen.sift_like(150_000, 128, seed=21)
    c16 = datagen.lloyd_centroids(x, 16, 256, iters=1, sample=4000, seed=5)
    c8 = datagen.lloyd_centroids(x, 8, 256, iters=1, sample=4000, seed=6)
    want16, _ = oracle.pq_assign(x, c16, threads=0)
    want8, _ = oracle.pq_assign(x, c8, threads=0)
    for cent, want in ((c16, want16), (c8, want8), (c16, want16), (c8, want8), (c16, want16)):
        got, _ = _assign(gpu, x, cent)
        assert np.array_equal(got, want), (got != want).sum()


def test_assign_nonfinite_rows(gpu, oracle):
    x = datagen.sift_like(300, 128, seed=2)
    cent = datagen.lloyd_centroids(x, 8, 256, iters=1, sample=300)
    x[5, 3] = np.nan
    x[9, 40] = np.inf
    x[11, 100] = 3e38
    want, _ = oracle.pq_assign(x, cent)
    got, _ = _assign(gpu, x, cent)
    assert np.array_equal(got, want)


def test_assign_small_and_ragged(gpu, oracle):
    x = datagen.deep_like(37, 96, seed=4)
    cent = datagen.lloyd_centroids(x, 16, 256, iters=1, sample=37)
    for n in (1, 2, 31, 32, 33, 37):
        want, _ = oracle.pq_assign(x[:n], cent)
        got, _ = _assign(gpu, x[:n], cent)
        assert np.array_equal(got, want), n


@pytest.mark.parametrize("kind", ["sift", "deep"])
def test_assign_k4096_vs_oracle(gpu, oracle, kind):
    """K = 4,096 (u16 codes, BASELINE configs[4]): the MFMA screening with centroid tiles
    streamed from L2 == the oracle, with the counts the call asked for, and the exact kernel
    agrees; first-index ties among duplicated centroids and non-finite rows too."""
    torch, codec, ctx = gpu
    n = 3001
    x = datagen.sift_like(n, 128, seed=51) if kind == "sift" else datagen.deep_like(n, 128, seed=52)
    rng = np.random.default_rng(53)
    rows = x[rng.choice(n, 2048, replace=False)].reshape(2048, 8, 16).transpose(1, 0, 2)
    cent = np.concatenate([rows, rows + rng.normal(0, 0.3, rows.shape)], axis=1)
    cent = np.ascontiguousarray(cent).astype(np.float32)          # (8, 4096, 16)
    cent[:, 4000:4096] = cent[:, 100:196]                          # duplicates: ties
    x[7, 5] = np.nan
    x[8, 60] = np.inf
    want, _ = oracle.pq_assign(x, cent, threads=0)
    counts = torch.zeros((8, 4096), dtype=torch.int32, device="cuda")
    got, rr = _assign(gpu, x, cent, 0, counts)
    got = got.view(np.uint16)                      # (torch keeps u16 codes as int16)
    assert np.array_equal(got, want.astype(np.uint16)), (got != want).sum()
    assert rr > 0
    assert np.array_equal(codec.counts_to_host(counts), oracle.histogram(want, 4096, False))
    got1, rr1 = _assign(gpu, x, cent, 1)
    assert np.array_equal(got1.view(np.uint16), want.astype(np.uint16)) and rr1 == 0


def test_assign_k_not_256_uses_exact_kernel(gpu, oracle):
    x = datagen.sift_like(500, 64, seed=9)
    for k in (16, 1000):
        cent = datagen.lloyd_centroids(x, 4, k, iters=1, sample=500)
        want, _ = oracle.pq_assign(x, cent)
        got, _ = _assign(gpu, x, cent)
        assert np.array_equal(got, want.astype(got.dtype).view(got.dtype)), k


def test_fused_histogram(gpu, oracle):
    torch, codec, ctx = gpu
    x = datagen.sift_like(3000, 128, seed=21)
    cent = datagen.lloyd_centroids(x, 8, 256, iters=1, sample=3000)
    counts = torch.zeros((8, 256), dtype=torch.int32, device="cuda")
    codes, _ = _assign(gpu, x, cent, 0, counts)
    assert np.array_equal(codec.counts_to_host(counts), oracle.histogram(codes, 256, False))


def test_error_and_reconstruct(gpu, oracle):
    torch, codec, ctx = gpu
    g = golden("pq_sift_n1000_m8_k256.npz")
    pq = codec.PQ(ctx, g["centroids"])
    xd = torch.from_numpy(g["x"]).cuda()
    cd = torch.from_numpy(g["codes"]).cuda()
    err = pq.error(xd, cd)
    want = oracle.compute_error(g["x"], g["centroids"], g["codes"])
    assert abs(err - want) <= 1e-12 * abs(want)
    rec = pq.reconstruct(cd).cpu().numpy()
    c = g["centroids"]
    ref = np.concatenate([c[i][g["codes"][:, i]] for i in range(8)], axis=1)
    assert np.array_equal(rec, ref)


def _init_from_rows(x, m, k, seed):
    rng = np.random.default_rng(seed)
    rows = rng.choice(x.shape[0], k, replace=False)
    ds = x.shape[1] // m
    return np.ascontiguousarray(x[rows].reshape(k, m, ds).transpose(1, 0, 2))


@pytest.mark.parametrize("n,d,m,k,iters", [(3000, 32, 4, 16, 5), (20000, 128, 8, 256, 3),
                                           (4000, 96, 16, 256, 2), (2500, 64, 8, 300, 2)])
def test_kmeans_train_vs_oracle(gpu, oracle, n, d, m, k, iters):
    """GPU Lloyd (fixed-point sums) equals the oracle's sequential restatement bit for bit."""
    torch, codec, ctx = gpu
    x = datagen.sift_like(n, d, seed=3) if d == 128 else \
        np.random.default_rng(4).normal(0, 1, (n, d)).astype(np.float32)
    init = _init_from_rows(x, m, k, 7)
    got = codec.kmeans_train(ctx, torch.from_numpy(x).cuda(), init, iters)
    want = oracle.kmeans(x, init, iters, threads=0)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_kmeans_train_reduces_error(gpu, oracle):
    torch, codec, ctx = gpu
    x = datagen.sift_like(20000, 128, seed=9)
    init = _init_from_rows(x, 8, 256, 1)
    xd = torch.from_numpy(x).cuda()
    errs = []
    for it in (0, 1, 4):
        c = codec.kmeans_train(ctx, xd, init, it)
        codes, _ = oracle.pq_assign(x, c, threads=0)
        errs.append(oracle.compute_error(x, c, codes))
    assert errs[0] > errs[1] > errs[2]


def test_cli_pq_encoder_trains_on_gpu(gpu, oracle, tmp_path):
    """pq_encoder without --centroids: seeded row init (the CLI's xorshift sampler), GPU
    training, then GPU assignment -- equal to the oracle's training from the same init."""
    import os
    import subprocess
    from conftest import ROOT
    x = datagen.sift_like(5000, 128, seed=2)
    datagen.write_fvecs(str(tmp_path / "x.fvecs"), x)
    bind = os.path.join(ROOT, "pq_huffman_amd", "bin")
    subprocess.run([os.path.join(bind, "pq_encoder"), str(tmp_path / "x.fvecs"),
                    str(tmp_path) + "/", "8", "--kmeans-iterations", "3"], check=True,
                   capture_output=True, timeout=300)
    state = 0x9E3779B97F4A7C15
    mask = (1 << 64) - 1
    rows = []
    for _ in range(256):                       # tools/pq_encoder.c rng_next
        state ^= (state << 13) & mask
        state ^= state >> 7
        state ^= (state << 17) & mask
        rows.append(state % 5000)
    init = np.ascontiguousarray(x[rows].reshape(256, 8, 16).transpose(1, 0, 2))
    want = oracle.kmeans(x, init, 3, threads=0)
    raw = (tmp_path / "pq_centroids.fvecsl").read_bytes()
    got = np.frombuffer(raw[8:], np.float32).reshape(8, 256, 16)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    codes_raw = (tmp_path / "pq_indices.bvecsl").read_bytes()
    want_codes, _ = oracle.pq_assign(x, want, threads=0)
    assert np.array_equal(np.frombuffer(codes_raw[8:], np.uint8).reshape(5000, 8), want_codes)


def test_pq_encode_streams_in_chunks(gpu, oracle, monkeypatch):
    """pq.h pq_encode (host pointers) on 7,777 rows through 1,000-row chunks -- two pinned
    buffers, so device memory holds two chunks -- equals the one-shot device assignment and
    the oracle (src/pq_encoder.c:43,58-80 reads 128K-row batches)."""
    import ctypes
    from pq_huffman_amd.capi import lib

    class CB(ctypes.Structure):   # pq.h centroids_codebook_t
        _fields_ = [("num_clusters", ctypes.c_int), ("num_dimensions", ctypes.c_int),
                    ("num_parts", ctypes.c_int), ("centroids_pool", ctypes.c_void_p),
                    ("centroids", ctypes.c_void_p)]

    monkeypatch.setenv("PQH_ENCODE_CHUNK", "1000")
    n = 7777
    x = datagen.sift_like(n, 128, seed=5)
    cent = np.ascontiguousarray(datagen.lloyd_centroids(x, 8, 256, iters=1, sample=4000), np.float32)
    cb = CB(256, 16, 8, cent.ctypes.data, None)
    codes = np.zeros((n, 8), np.uint8)
    assert lib().pq_encode(ctypes.byref(cb), x.ctypes.data, n, 128, codes.ctypes.data) == 0
    one_shot, _ = _assign(gpu, x, cent)
    assert np.array_equal(codes, one_shot)
    want, _ = oracle.pq_assign(x, cent, threads=0)
    assert np.array_equal(codes, want)


def _cb_struct():
    import ctypes

    class CB(ctypes.Structure):   # pq.h centroids_codebook_t
        _fields_ = [("num_clusters", ctypes.c_int), ("num_dimensions", ctypes.c_int),
                    ("num_parts", ctypes.c_int), ("centroids_pool", ctypes.c_void_p),
                    ("centroids", ctypes.c_void_p)]
    return CB


def _row_reader(x):
    """a pq_rows_fn over a numpy array, counting the rows it hands out"""
    import ctypes
    seen = {"rows": 0, "max_chunk": 0}
    fn_t = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong,
                            ctypes.c_void_p)

    def read(_user, row0, rows, dst):
        ctypes.memmove(dst, x[row0:row0 + rows].ctypes.data, rows * x.shape[1] * 4)
        seen["rows"] += rows
        seen["max_chunk"] = max(seen["max_chunk"], rows)
        return 0
    return fn_t(read), seen


def test_streamed_error_and_training_equal_one_shot(gpu, oracle):
    """pq_compute_error_rows / pq_train_rows (pq.h) over 1,024-row chunks -- device memory two
    chunks -- equal the one-shot device passes bit for bit: the error's 256-row partials are
    summed in row order, the k-means sums are exact fixed-point integers
    (src/pq_encoder.c:82-119 reads 128K-row batches; :265-269 one slice at a time)."""
    import ctypes
    from pq_huffman_amd.capi import lib
    torch, codec, ctx = gpu
    n = 7777
    x = datagen.sift_like(n, 128, seed=11)
    init = _init_from_rows(x, 8, 256, 3)
    CB = _cb_struct()
    # training: 3 iterations streamed vs the one-shot device trainer vs the oracle
    cent = np.ascontiguousarray(init.copy(), np.float32)
    cb = CB(256, 16, 8, cent.ctypes.data, None)
    rd, seen = _row_reader(x)
    assert lib().pq_train_rows(ctypes.byref(cb), 128, n, rd, None, 3, 1024) == 0
    assert seen["max_chunk"] == 1024 and seen["rows"] == 4 * n   # absmax + 3 iterations
    one = codec.kmeans_train(ctx, torch.from_numpy(x).cuda(), init, 3)
    assert np.array_equal(cent.view(np.uint32), one.view(np.uint32))
    assert np.array_equal(cent.view(np.uint32), oracle.kmeans(x, init, 3, threads=0).view(np.uint32))
    # error of the trained codebook's codes: streamed vs one-shot vs the oracle
    codes, _ = oracle.pq_assign(x, cent, threads=0)
    rd2, seen2 = _row_reader(x)
    err = ctypes.c_double()
    assert lib().pq_compute_error_rows(ctypes.byref(cb), 128, n, rd2, None, codes.ctypes.data,
                                       1024, ctypes.byref(err)) == 0
    assert seen2["max_chunk"] == 1024 and seen2["rows"] == n
    pq = codec.PQ(ctx, cent)
    one_err = pq.error(torch.from_numpy(x).cuda(), torch.from_numpy(codes).cuda())
    assert err.value == one_err
    want = oracle.compute_error(x, cent, codes)
    assert abs(err.value - want) <= 1e-12 * abs(want)


def test_cli_pq_encoder_compute_error_streams(gpu, oracle, tmp_path):
    """pq_encoder --compute-error on an input of several chunks (PQH_ENCODE_CHUNK=1024): the
    training, the codes and the appended pq_error equal the one-shot passes on the same rows."""
    import os
    import subprocess
    from conftest import ROOT
    torch, codec, ctx = gpu
    n = 6000
    x = datagen.sift_like(n, 128, seed=12)
    datagen.write_fvecs(str(tmp_path / "x.fvecs"), x)
    bind = os.path.join(ROOT, "pq_huffman_amd", "bin")
    env = dict(os.environ, PQH_ENCODE_CHUNK="1024")
    subprocess.run([os.path.join(bind, "pq_encoder"), str(tmp_path / "x.fvecs"),
                    str(tmp_path) + "/", "8", "--kmeans-iterations", "2", "--compute-error"],
                   check=True, capture_output=True, timeout=300, env=env)
    state = 0x9E3779B97F4A7C15
    mask = (1 << 64) - 1
    rows = []
    for _ in range(256):                       # tools/pq_encoder.c rng_next
        state ^= (state << 13) & mask
        state ^= state >> 7
        state ^= (state << 17) & mask
        rows.append(state % n)
    init = np.ascontiguousarray(x[rows].reshape(256, 8, 16).transpose(1, 0, 2))
    cent = codec.kmeans_train(ctx, torch.from_numpy(x).cuda(), init, 2)
    got = np.frombuffer((tmp_path / "pq_centroids.fvecsl").read_bytes()[8:], np.float32)
    assert np.array_equal(got.view(np.uint32), cent.reshape(-1).view(np.uint32))
    codes = np.frombuffer((tmp_path / "pq_indices.bvecsl").read_bytes()[8:], np.uint8).reshape(n, 8)
    want_codes, _ = oracle.pq_assign(x, cent, threads=0)
    assert np.array_equal(codes, want_codes)
    one_err = codec.PQ(ctx, cent).error(torch.from_numpy(x).cuda(),
                                        torch.from_numpy(codes.copy()).cuda())
    assert (tmp_path / "pq_error").read_text() == "%f\n" % one_err
