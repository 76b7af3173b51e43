"""Tree-ordered context coding (huffman_encoder --tree mst.tree; huffman_encoder.c:240-286,
:321-375; mst.c:253-490).

CPU: the oracle against the fixtures the reference's own binaries produced
(oracle/gen_golden.py tree: huffman_encoder --tree / huffman_decoder --tree on seeded
forests in the mst.tree layout), and the library's host DFS/traverser walk against the
oracle.  GPU: pqh_tree_gather + pqh_histogram_tree + GPU code tables + pqh_encode_tree_write
byte-identical to the reference files, and at larger sizes to the oracle (plus an oracle
decode round trip)."""
import numpy as np
import pytest

from conftest import golden
import datagen

CASES = ["tree_m8_n1000", "tree_m16_n300", "tree_m8_n64_forest"]
FILES = ["huffman_codebooks", "huffman_indices", "huffman_children_codebooks",
         "huffman_children"]


def _oracle_files(oracle, codes, targets, counts):
    vert, nch, _ = oracle.tree_order(len(counts), targets, counts)
    par = oracle.tree_parents(nch, vert)
    cbs = oracle.tree_codebooks(codes, vert, par)
    stream, bits = oracle.tree_encode(codes, vert, par, cbs)
    _, ccb = oracle.children_codebook(nch)
    return vert, nch, par, cbs, stream, ccb


def _children_stream(oracle, ccb, nch):
    codes = np.ascontiguousarray(nch.reshape(-1, 1).astype(np.uint16 if ccb.k > 256 else np.uint8))
    return oracle.encode(codes, ccb)[0]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mode", ["tree_nosort", "tree_sort"])
def test_oracle_tree_vs_reference_files(oracle, case, mode):
    g = golden(f"huff_{case}.npz")
    codes = g["input"]
    if mode == "tree_sort":          # the CLI sorts first by default (huffman_encoder.c:313)
        codes = oracle.sort_rows(codes)
    vert, nch, par, cbs, stream, ccb = _oracle_files(oracle, codes, g["targets"], g["counts"])
    assert oracle.codebooks_file(cbs) == g[mode + "__huffman_codebooks"].tobytes()
    assert np.uint64(len(codes)).tobytes() + stream == g[mode + "__huffman_indices"].tobytes()
    assert oracle.serialize(ccb.k, False, ccb.lens[0], ccb.codes[0]) == \
        g[mode + "__huffman_children_codebooks"].tobytes()
    assert _children_stream(oracle, ccb, nch) == g[mode + "__huffman_children"].tobytes()
    # the reference decoder emits rows in stream (DFS) order
    np.testing.assert_array_equal(g[mode + "__decoded"], codes[vert])
    np.testing.assert_array_equal(oracle.tree_decode(stream, len(codes), codes.shape[1], cbs, nch),
                                  codes[vert])


@pytest.mark.parametrize("n,roots,seed", [(1, 1, 1), (2, 1, 2), (1000, 3, 3), (5000, 40, 4),
                                          (64, 64, 5), (20000, 1, 6)])
def test_library_tree_order_vs_oracle(oracle, n, roots, seed):
    from pq_huffman_amd import codec
    targets, counts = datagen.random_forest(n, roots=roots, seed=seed)
    vert, nch, par, nroots = codec.tree_order(targets, counts)
    ov, onch, oroots = oracle.tree_order(n, targets, counts)
    np.testing.assert_array_equal(vert, ov)
    np.testing.assert_array_equal(nch, onch)
    assert nroots == oroots == roots
    np.testing.assert_array_equal(par, oracle.tree_parents(onch, ov))
    assert sorted(vert.tolist()) == list(range(n))
    assert (par < 0).sum() == roots


def test_library_tree_order_rejects_malformed():
    from pq_huffman_amd import codec
    from pq_huffman_amd.capi import PqhError
    targets, counts = datagen.random_forest(50, roots=2, seed=7)
    with pytest.raises(PqhError):             # edge count disagrees with the adjacency sizes
        codec.tree_order(targets[:-1], counts)
    bad = targets.copy()
    bad[0] = 50                               # target outside the vertices
    with pytest.raises(PqhError):
        codec.tree_order(bad, counts)
    # a target repeated in one list counts twice before the push (mst.c:322-333), so the
    # child sum breaks the reference's assert (mst.c:357)
    with pytest.raises(PqhError):
        codec.tree_order(np.array([1, 1], np.uint32), np.array([2, 0, 0], np.int32))


@pytest.mark.parametrize("targets,counts", [
    ([1, 2, 0, 2, 0, 1], [2, 2, 2]),          # both directions and a cycle: back edges skipped
    ([0, 1, 1, 0], [2, 1, 1]),                # self loops on a root and on a child
    ([3, 2, 1, 0], [1, 1, 1, 1]),             # two trees whose second root is not the lowest id
])
def test_library_tree_order_back_edges_vs_oracle(oracle, targets, counts):
    from pq_huffman_amd import codec
    t, c = np.array(targets, np.uint32), np.array(counts, np.int32)
    vert, nch, par, nroots = codec.tree_order(t, c)
    ov, onch, oroots = oracle.tree_order(len(c), t, c)
    np.testing.assert_array_equal(vert, ov)
    np.testing.assert_array_equal(nch, onch)
    assert nroots == oroots


def test_tree_file_roundtrip(tmp_path):
    from pq_huffman_amd import codec
    targets, counts = datagen.random_forest(300, roots=4, seed=8)
    p = str(tmp_path / "mst.tree")
    datagen.write_tree(p, 300, targets, counts)
    n, t2, c2 = codec.load_tree(p)
    assert n == 300
    np.testing.assert_array_equal(t2, targets)
    np.testing.assert_array_equal(c2, counts)


# ---------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def gpu():
    import torch
    from pq_huffman_amd import codec
    assert torch.cuda.is_available(), "GPU tests need the MI355X (no fallback path)"
    ctx = codec.Context(0)
    yield ctx
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("mode", ["tree_nosort", "tree_sort"])
def test_gpu_tree_encode_vs_reference_files(gpu, oracle, case, mode):
    import torch
    from pq_huffman_amd import codec
    g = golden(f"huff_{case}.npz")
    codes = g["input"]
    d = torch.from_numpy(codes).cuda()
    if mode == "tree_sort":
        codec.sort_rows(gpu, d)
    enc = codec.tree_encode(gpu, d, g["targets"], g["counts"])
    files = codec.tree_files(enc)
    for f in FILES:
        assert files[f + ".bin"] == g[mode + "__" + f].tobytes(), f
    np.testing.assert_array_equal(codec.tree_decode(gpu, enc).cpu().numpy(),
                                  g[mode + "__decoded"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,roots", [(200_000, 8, 17), (50_000, 16, 1), (1_000_000, 8, 1000)])
def test_gpu_tree_encode_vs_oracle_roundtrip(gpu, oracle, n, m, roots):
    import torch
    from pq_huffman_amd import codec
    codes = datagen.skewed_codes(n, m, 256, seed=n + m)
    targets, counts = datagen.random_forest(n, roots=roots, seed=roots)
    enc = codec.tree_encode(gpu, torch.from_numpy(codes).cuda(), targets, counts)
    vert, nch, _ = oracle.tree_order(n, targets, counts)
    par = oracle.tree_parents(nch, vert)
    cbs = oracle.tree_codebooks(codes, vert, par)
    stream, bits = oracle.tree_encode(codes, vert, par, cbs)
    assert enc.bits == bits
    got = enc.stream[:enc.nbytes].cpu().numpy().tobytes()
    assert got == stream
    np.testing.assert_array_equal(oracle.tree_decode(got, n, m, cbs, enc.num_children),
                                  codes[enc.vertices])
    assert enc.children.stream[:enc.children.nbytes].cpu().numpy().tobytes() == \
        _children_stream(oracle, oracle.children_codebook(nch)[1], nch)
    # GPU tree decode (chunked, with the encoder's sidecar) returns the stream-order rows
    for c in (16, 7, 64):
        e2 = enc if c == 16 else codec.tree_encode(gpu, torch.from_numpy(codes).cuda(), targets,
                                                   counts, chunk_vectors=c)
        dec = codec.tree_decode(gpu, e2).cpu().numpy()
        np.testing.assert_array_equal(dec, codes[enc.vertices])


@pytest.mark.gpu
@pytest.mark.parametrize("cut", [1, 4, 1000])
def test_gpu_tree_decode_rejects_truncated_stream(gpu, cut):
    """A stream shorter than the encoder's sidecar says (a truncated huffman_indices.bin)
    is reported as corrupt, never decoded into garbage rows."""
    import torch
    from pq_huffman_amd import codec
    from pq_huffman_amd.capi import PqhError
    n, m = 20_000, 8
    codes = datagen.skewed_codes(n, m, 256, seed=3)
    targets, counts = datagen.random_forest(n, roots=5, seed=4)
    enc = codec.tree_encode(gpu, torch.from_numpy(codes).cuda(), targets, counts)
    dec = codec.tree_decode(gpu, enc).cpu().numpy()          # exact length: fine
    np.testing.assert_array_equal(dec, codes[enc.vertices])
    with pytest.raises(PqhError):
        codec.tree_decode(gpu, enc, stream_bytes=enc.nbytes - cut)
    dec = codec.tree_decode(gpu, enc).cpu().numpy()          # the next decode is clean
    np.testing.assert_array_equal(dec, codes[enc.vertices])


@pytest.mark.gpu
def test_gpu_tree_gather_reports_bad_ids(gpu):
    import torch
    from pq_huffman_amd import codec
    from pq_huffman_amd.capi import lib
    n, m = 1000, 8
    codes = torch.zeros((n, m), dtype=torch.uint8, device="cuda")
    vert = torch.arange(n, dtype=torch.int32, device="cuda")
    vert[5] = n + 3
    par = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    rows = torch.empty_like(codes)
    prev = torch.empty((n, m), dtype=torch.int16, device="cuda")
    assert lib().pqh_tree_gather(gpu.ptr, codes.data_ptr(), n, m, 256, vert.data_ptr(),
                                 par.data_ptr(), rows.data_ptr(), prev.data_ptr()) == 0
    assert lib().pqh_tree_status(gpu.ptr) != 0
    assert lib().pqh_tree_status(gpu.ptr) == 0      # the flag is cleared after a report


@pytest.mark.parametrize("n,roots,c", [(1000, 3, 64), (5000, 40, 7), (20000, 1, 64), (1, 1, 4)])
def test_tree_ext_index_vs_oracle(oracle, n, roots, c):
    """The decode sidecar index: parent positions equal the oracle traverser's, and the ext
    list is exactly the rows whose context precedes their chunk, in row order."""
    from pq_huffman_amd import codec
    targets, counts = datagen.random_forest(n, roots=roots, seed=n + c)
    _, nch, _ = oracle.tree_order(n, targets, counts)
    pp, eo, ep = codec.tree_ext_index(nch, c)
    np.testing.assert_array_equal(pp, oracle.tree_parents(nch))
    rows = np.arange(n)
    ext = (pp >= 0) & (pp < rows - rows % c)
    np.testing.assert_array_equal(ep, pp[ext])
    np.testing.assert_array_equal(eo[:-1], np.concatenate([[0], np.cumsum(ext)])[rows[::c]])
    assert eo[-1] == ext.sum()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["device", "host"])
@pytest.mark.parametrize("mode,flags", [("tree_nosort", ["--no-sort"]), ("tree_sort", [])])
def test_cli_encoder_tree_matches_reference_files(tmp_path, mode, flags, order):
    """huffman_encoder --tree (pqh_encode_tree_files) writes the reference's six files, with
    the device tree order and with the host walk (PQH_TREE_ORDER=host)."""
    import os
    import subprocess
    from conftest import ROOT
    g = golden("huff_tree_m8_n1000.npz")
    pqdir, out = tmp_path / "pq", tmp_path / "out"
    pqdir.mkdir()
    out.mkdir()
    datagen.write_vecsl(str(pqdir / "pq_indices.bvecsl"), g["input"])
    tree = tmp_path / "mst.tree"
    datagen.write_tree(str(tree), 1000, g["targets"], g["counts"])
    r = subprocess.run([os.path.join(ROOT, "pq_huffman_amd", "bin", "huffman_encoder"),
                        str(pqdir) + "/", str(out) + "/", "8", "--tree", str(tree)] + flags,
                       capture_output=True, text=True,
                       env=dict(os.environ, PQH_TREE_ORDER=order))
    assert r.returncode == 0, r.stdout + r.stderr
    for f in FILES + ["huffman_stats", "huffman_children_stats"]:
        ext = ".txt" if f.endswith("stats") else ".bin"
        assert (out / (f + ext)).read_bytes() == g[mode + "__" + f].tobytes(), f
    # huffman_decoder --tree: the GPU decode (with the sidecar) gives the reference's rows
    dec = tmp_path / "dec.bin"
    r = subprocess.run([os.path.join(ROOT, "pq_huffman_amd", "bin", "huffman_decoder"),
                        str(out) + "/", "--tree", "--output-file", str(dec), "--check-file",
                        str(pqdir / "pq_indices.bvecsl")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert dec.read_bytes() == g[mode + "__decoded"].tobytes()
    (out / "huffman_tree_chunks.bin").unlink()      # no sidecar: refused, not mis-decoded
    r = subprocess.run([os.path.join(ROOT, "pq_huffman_amd", "bin", "huffman_decoder"),
                        str(out) + "/", "--tree", "--output-file", str(dec)],
                       capture_output=True, text=True)
    assert r.returncode != 0


# ------------------------------------------------- device DFS order (Euler tour)
def _path_forest(n, seed):
    """One path through a random permutation of the ids (depth n - 1)."""
    rng = np.random.default_rng(seed)
    p = rng.permutation(n)
    adj = [[] for _ in range(n)]
    for a, b in zip(p[:-1], p[1:]):
        adj[a].append(b)
        adj[b].append(a)
    return (np.array([t for a in adj for t in a], np.uint32),
            np.array([len(a) for a in adj], np.int32))


def _star_forest(n, centre):
    adj = [[] for _ in range(n)]
    for v in range(n):
        if v != centre:
            adj[centre].append(v)
            adj[v].append(centre)
    return (np.array([t for a in adj for t in a], np.uint32),
            np.array([len(a) for a in adj], np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,n,roots", [
    ("random", 1, 1), ("random", 2, 1), ("random", 64, 64), ("random", 1000, 3),
    ("random", 200_000, 17), ("random", 1_000_000, 1000), ("random", 300_000, 1),
    ("path", 100_000, 1), ("star", 50_000, 1), ("two", 4, 2)])
def test_gpu_tree_order_device_vs_host(gpu, shape, n, roots):
    """pqh_tree_order_device equals the host walk (tree_collect_vertices_dfs + traverser
    parents): preorder from each tree's lowest id, children in reverse adjacency order."""
    from pq_huffman_amd import codec
    if shape == "random":
        targets, counts = datagen.random_forest(n, roots=roots, seed=n + roots)
    elif shape == "path":
        targets, counts = _path_forest(n, seed=5)
    elif shape == "star":
        targets, counts = _star_forest(n, centre=n // 3)
    else:                                      # second tree's root is not the lowest id
        targets, counts = np.array([3, 2, 1, 0], np.uint32), np.array([1, 1, 1, 1], np.int32)
    vert, nch, par, nroots = codec.tree_order(targets, counts)
    got = codec.tree_order_device(gpu, targets, counts)
    assert got is not None
    dv, dn, dp, droots = got
    assert droots == nroots == roots
    np.testing.assert_array_equal(dv.cpu().numpy().view(np.uint32), vert)
    np.testing.assert_array_equal(dn.cpu().numpy(), nch)
    np.testing.assert_array_equal(dp.cpu().numpy(), par)


@pytest.mark.gpu
@pytest.mark.parametrize("targets,counts", [
    ([1, 2, 0, 2, 0, 1], [2, 2, 2]),          # a cycle
    ([0, 1, 1, 0], [2, 1, 1]),                # self loops
    ([1, 1], [2, 0, 0]),                      # a repeated edge stored in one direction
    ([1, 2, 0, 2, 0, 1, 3, 2], [2, 2, 3, 1]),  # a triangle 0-1-2 with a pendant edge 2-3
])
def test_gpu_tree_order_device_declines_non_forests(gpu, targets, counts):
    """A graph that is not a forest is declined (None), and the encoder's host walk takes it."""
    from pq_huffman_amd import codec
    t, c = np.array(targets, np.uint32), np.array(counts, np.int32)
    assert codec.tree_order_device(gpu, t, c) is None


@pytest.mark.gpu
def test_gpu_tree_order_device_large_cycle(gpu):
    """A forest plus one long cycle (every vertex has an edge down into it from the tour
    pass, but the edge count exceeds a forest's): declined."""
    from pq_huffman_amd import codec
    n = 10_000
    adj = [[] for _ in range(n)]
    for v in range(n):
        w = (v + 1) % n
        adj[v].append(w)
        adj[w].append(v)
    t = np.array([x for a in adj for x in a], np.uint32)
    c = np.array([len(a) for a in adj], np.int32)
    assert codec.tree_order_device(gpu, t, c) is None


@pytest.mark.gpu
def test_gpu_tree_order_device_rejects_bad_counts(gpu):
    from pq_huffman_amd import codec
    from pq_huffman_amd.capi import PqhError
    targets, counts = datagen.random_forest(50, roots=2, seed=7)
    with pytest.raises(PqhError):             # counts do not sum to the edge count
        codec.tree_order_device(gpu, targets[:-1], counts)
    bad = counts.copy()
    bad[0], bad[1] = bad[0] + 3, -3           # right sum, a negative count
    with pytest.raises(PqhError):
        codec.tree_order_device(gpu, targets, bad)
    bad_t = targets.copy()
    bad_t[0] = 50                             # target outside the vertices: not a forest
    assert codec.tree_order_device(gpu, bad_t, counts) is None


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,c", [("forest", 1, 16), ("forest", 2, 1), ("forest", 1000, 7),
                                      ("forest", 200_000, 16), ("forest", 1_000_000, 64),
                                      ("path", 100_000, 16), ("star", 50_000, 16),
                                      ("arbitrary", 5000, 3), ("arbitrary", 300_000, 16),
                                      ("wide", 70_000, 16)])
@pytest.mark.parametrize("width", [1, 2, 4])
def test_gpu_tree_ext_index_device_vs_host(gpu, kind, n, c, width):
    """The decoder's traverser index on the device (pqh_tree_ext_index_device) equals the
    host walk (pqh_tree_ext_index) -- for forests' DFS child counts and for arbitrary counts
    (truncated trees, slots left open at the end), read as u8 / u16 / i32."""
    import torch
    from pq_huffman_amd import codec
    rng = np.random.default_rng(n + c + width)
    if kind == "forest":
        t, cnt = datagen.random_forest(n, roots=max(1, n // 5000), seed=n)
        nch = codec.tree_order(t, cnt)[1]
    elif kind == "path":
        nch = codec.tree_order(*_path_forest(n, seed=3))[1]
    elif kind == "star":
        nch = codec.tree_order(*_star_forest(n, centre=7))[1]
    elif kind == "wide":                       # child counts past 255 (u16 / i32 only)
        nch = np.zeros(n, np.int32)
        nch[::1000] = rng.integers(0, 3000, len(nch[::1000]))
    else:
        nch = rng.integers(0, 4, n).astype(np.int32)
        nch[rng.random(n) < 0.55] = 0
    nch = np.asarray(nch, np.int32)
    if width == 1 and nch.max() > 255:
        pytest.skip("u8 counts cannot hold this forest's widest vertex")
    pp, eo, ep = codec.tree_ext_index(nch, c)
    dt = {1: torch.uint8, 2: torch.int16, 4: torch.int32}[width]
    d = torch.from_numpy(nch.astype({1: np.uint8, 2: np.uint16, 4: np.int32}[width])
                         .view({1: np.uint8, 2: np.int16, 4: np.int32}[width])).cuda()
    assert d.dtype == dt
    dpp, deo, ext, dep = codec.tree_ext_index_device(gpu, d, c, positions=True)
    assert ext == len(ep)
    np.testing.assert_array_equal(dpp.cpu().numpy(), pp)
    np.testing.assert_array_equal(deo.cpu().numpy(), eo)
    np.testing.assert_array_equal(dep.cpu().numpy(), ep)
