"""The forest builder's CLIs (pq_huffman_amd/bin/compute_nn_fast, mst_builder) against the
reference-produced fixtures: nn_indices.ivecsl / nn_dist.fvecsl equal the reference heap
merge's output (tests/golden/forest_*.npz), blocks_stat.txt lists the reference block sizes,
a --blocks-info-cache written by the first run is read back by the second (same files), and
mst_builder's mst.tree, stats.json and stats_num_children.json are byte-identical to the
reference mst_builder's for three take / penalty settings (mst_builder.c:98-131)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden
import datagen

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "pq_huffman_amd", "bin")
CASES = ["forest_sift_n1200_d16.npz", "forest_deep_n800_d12.npz"]


def _run(args):
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    return r.stdout


def _rows(path, dtype):
    raw = open(path, "rb").read()
    n, cols = np.frombuffer(raw[:8], np.uint32)
    return np.frombuffer(raw[8:], dtype).reshape(n, cols)


@pytest.mark.parametrize("name", CASES)
def test_compute_nn_fast_cli(tmp_path, name):
    g = golden(name)
    fv = str(tmp_path / "x.fvecs")
    datagen.write_fvecs(fv, g["x"])
    cache = str(tmp_path / "blocks_info_cache.dat")
    for run in range(2):   # the second run reads the geometry from the cache
        out = str(tmp_path / f"out{run}") + "/"
        os.makedirs(out)
        _run([os.path.join(BIN, "compute_nn_fast"), fv, out, str(int(g["num_nn"])),
              "--num-dims", str(int(g["num_split"])), "--num-blocks-per-dim",
              str(int(g["blocks_per_dim"])), "--block-overlap-fraction", str(float(g["overlap"])),
              "--blocks-info-cache", cache, "--with-blocks-stat", "--num-threads", "4",
              "--no-delete-temp-file"])
        np.testing.assert_array_equal(_rows(out + "nn_indices.ivecsl", np.uint32), g["nn_idx"])
        np.testing.assert_array_equal(_rows(out + "nn_dist.fvecsl", np.float32), g["nn_dist"])
        sizes = [int(s) for s in open(out + "blocks_stat.txt").read().split()]
        assert sizes == list(g["member"].sum(axis=1))
    raw = open(cache, "rb").read()   # blocks_info_save_file layout (fast_nn_blocks_info.c:124-137)
    ns, nb = int(g["num_split"]), int(g["blocks_per_dim"])
    assert len(raw) == 4 + 8 + 4 + 8 + ns * (4 + 8 + 8 * nb)
    assert np.frombuffer(raw[:4], np.int32)[0] == ns


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("tag,take,pen", [("t5_p0", 5, "0"), ("t3_p2.5", 3, "2.5"),
                                          ("tall_pinf", None, "inf")])
def test_mst_builder_cli(tmp_path, name, tag, take, pen):
    g = golden(name)
    nd = str(tmp_path / "nn") + "/"
    pqd = str(tmp_path / "pq") + "/"
    out = str(tmp_path / "out") + "/"
    for d in (nd, pqd, out):
        os.makedirs(d)
    n, nn = g["nn_idx"].shape
    for fn, a in (("nn_indices.ivecsl", g["nn_idx"]), ("nn_dist.fvecsl", g["nn_dist"])):
        with open(nd + fn, "wb") as f:
            f.write(np.array([n, nn], np.uint32).tobytes() + a.tobytes())
    datagen.write_vecsl(pqd + "pq_indices.bvecsl", g["pq"])
    _run([os.path.join(BIN, "mst_builder"), nd, out, str(take or nn), "--pq-template", pqd,
          "--pq-penalty", pen])
    assert open(out + "mst.tree", "rb").read() == g[f"tree_{tag}"].tobytes()
    assert open(out + "stats.json", "rb").read() == g[f"stats_{tag}"].tobytes()
    assert open(out + "stats_num_children.json", "rb").read() == g[f"stats_children_{tag}"].tobytes()
