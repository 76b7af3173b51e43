"""The forest builder's oracle (oracle/pqh_oracle.c orc_knn_* / orc_mst) against fixtures
the REFERENCE produced (oracle/gen_golden.py forest): compute_nn_fast's block geometry
(blocks_info_init, fast_nn_blocks_info.c:94-112) and membership (is_vector_in_block,
:187-239), its heap merge of the in-block lists (fast_nn_heap_push/_sort,
fast_nn_temp_file.c:11-63), and mst_builder's mst.tree (mst.c:80-265) for three take /
PQ-penalty settings.  The in-block lists (yael's knn_full_thread in the reference) are the
oracle's own definition: parity unpinned at that call, so the fixture stores them as the
push log and the test checks the oracle reproduces them."""
import numpy as np
import pytest

from conftest import golden

CASES = ["forest_sift_n1200_d16.npz", "forest_deep_n800_d12.npz"]
TREES = [("t5_p0", 5, 0.0), ("t3_p2.5", 3, 2.5), ("tall_pinf", None, float("inf"))]


@pytest.mark.parametrize("name", CASES)
def test_geometry_and_membership(oracle, name):
    g = golden(name)
    st, en = oracle.knn_blocks_info(g["x"], int(g["num_split"]), int(g["blocks_per_dim"]),
                                    float(g["overlap"]))
    np.testing.assert_array_equal(st, g["starts"])
    np.testing.assert_array_equal(en, g["ends"])
    mem = oracle.knn_members(g["x"], st, en)
    for b, rows in enumerate(mem):
        np.testing.assert_array_equal(rows, np.nonzero(g["member"][b])[0])


@pytest.mark.parametrize("name", CASES)
def test_knn_merge_matches_reference_heap(oracle, name):
    g = golden(name)
    idx, dist, sizes, (lr, li, ld) = oracle.knn_fast(g["x"], int(g["num_nn"]), g["starts"],
                                                     g["ends"], log=True)
    np.testing.assert_array_equal(sizes, g["member"].sum(axis=1))
    np.testing.assert_array_equal(lr, g["push_row"])     # self-generated (definition)
    np.testing.assert_array_equal(li, g["push_idx"])
    np.testing.assert_array_equal(ld, g["push_dist"])
    np.testing.assert_array_equal(idx, g["nn_idx"])      # the reference's merge
    np.testing.assert_array_equal(dist, g["nn_dist"])
    i2, d2, _ = oracle.knn_fast(g["x"], int(g["num_nn"]), g["starts"], g["ends"])   # threaded
    np.testing.assert_array_equal(i2, idx)
    np.testing.assert_array_equal(d2, dist)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("tag,take,pen", TREES)
def test_mst_matches_reference_mst_builder(oracle, name, tag, take, pen):
    g = golden(name)
    take = take or int(g["num_nn"])
    tg, cn = oracle.mst(g["nn_idx"], g["nn_dist"], take, g["pq"], pen)
    assert oracle.tree_file(len(g["x"]), tg, cn) == g[f"tree_{tag}"].tobytes()
