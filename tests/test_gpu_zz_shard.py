"""The library's multi-GPU encode (pqh_shard_encode via shard.shard_encode) with two ranks
on one GPU (gloo hooks, fresh child processes): the stitched stream (pqh_shard_stitch) and
the global histogram must equal the oracle's one-shot results over all ranks' rows
(huffman_encoder.c:139-238), for even shards, a shard with no rows, and the slices of the
distributed sort (whose ragged halo also goes through shard.halo_ragged)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, run_fail_msg

pytestmark = pytest.mark.gpu


# torchrun's own c10d store binds port 0 and the ranks reuse it (TORCHELASTIC_USE_AGENT_STORE):
# no port is picked here and released before the launcher binds it.
_LAUNCH = ["--standalone", "--local-addr=127.0.0.1"]


@pytest.mark.parametrize("case,mode", [("even", "ctx"), ("even", "noctx"), ("ragged", "ctx"),
                                       ("sort", "ctx"), ("parts", "ctx"), ("parts", "noctx"),
                                       ("parts_ragged", "ctx")])
def test_two_rank_library_shard_encode(oracle, tmp_path, case, mode):
    dump = tmp_path / "shard.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           *_LAUNCH,
           os.path.join(ROOT, "tests", "shard_worker.py"), "--case", case, "--mode", mode,
           "--out", str(dump)]
    r = subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, run_fail_msg(r)
    d = np.load(dump, allow_pickle=False)
    rows = d["rows"]
    ctxm = mode == "ctx"
    if case == "sort":   # the slices in rank order are the stable strncmp-key sort of all rows
        import datagen
        allc = datagen.skewed_codes(20011, 8, 256, seed=77)
        allc[np.random.default_rng(3).random(allc.shape) < 0.2] = 0
        np.testing.assert_array_equal(rows, oracle.sort_rows(allc))
    np.testing.assert_array_equal(d["counts"].astype(np.int64),
                                  oracle.histogram(rows, 256, ctxm))
    want, bits = oracle.encode(rows, oracle.build_codebooks(rows, 256, ctxm))
    assert int(d["total"]) == bits
    assert d["stream"].tobytes() == want


def test_two_rank_library_shard_encode_one_rank_fails(tmp_path):
    """A local failure on rank 1 (an output buffer too small) must not leave rank 0 waiting
    in a collective: rank 1 gets its error, rank 0 PQH_ERR_REMOTE from pqh_shard_status."""
    dump = tmp_path / "shard.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           *_LAUNCH,
           os.path.join(ROOT, "tests", "shard_worker.py"), "--case", "fail", "--mode", "ctx",
           "--out", str(dump)]
    r = subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, run_fail_msg(r)
    assert int(np.load(dump, allow_pickle=False)["failed"]) == 1
