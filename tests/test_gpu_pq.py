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
                                      ("sift", 128, 16), ("sift", 128, 32), ("sift", 64, 4)])
def test_assign_vs_oracle_random(gpu, oracle, kind, d, m):
    n = 6001  # not a multiple of 32
    x = datagen.sift_like(n, d, seed=11) if kind == "sift" else datagen.deep_like(n, d, seed=12)
    cent = datagen.lloyd_centroids(x, m, 256, iters=2, sample=4000, seed=3)
    want, _ = oracle.pq_assign(x, cent, threads=0)
    got, rr = _assign(gpu, x, cent, 0)
    assert np.array_equal(got, want), (got != want).sum()
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
