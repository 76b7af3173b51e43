"""bench.py itself, run as a child process, against the oracle: the multi-rank schedule on one
GPU (gloo process group, every rank on cuda:0) -- the library's two-phase pqh_shard_encode, or
the Python composition (halo all-gather, histogram all-reduce, device bit offsets,
encode_write_at) -- whose shards' streams stitched on rank 0 must equal the oracle's one-shot
stream over all ranks' rows (huffman_encoder.c:207-238 over the concatenated input); the
multi-rank pipeline over RCCL with one rank; and the one-rank headline schedule itself.  Every
run dumps its rows and centroids, so the codes are checked against the oracle's assignment
too, and every rank must exit cleanly (status 0, no signal at teardown)."""
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


def _check_assignment(oracle, d):
    """the ranks' part-major assignment (pqh_pq_assign_parts, the bench's timed kernel) equals
    the oracle's fp32 first-minimum assignment of the same rows (src/pq_encoder.c:270-272)"""
    want, _ = oracle.pq_assign(d["x"], d["cent"], threads=0)
    bad = int((d["codes"] != want).sum())
    assert bad == 0, f"{bad} PQ codes differ from the oracle"


@pytest.mark.parametrize("path", ["library", "python"])
@pytest.mark.parametrize("mode", ["ctx", "noctx"])
def test_two_rank_rehearsal_stitched_stream(oracle, tmp_path, mode, path):
    """path library: the bench's default world > 1 schedule through the C ABI
    (pqh_shard_encode_tables on the table lane, pqh_shard_encode_write on the encode stream,
    torch.distributed hooks); python: the same steps composed in shard.py."""
    dump = tmp_path / "dump.npz"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           *_LAUNCH,
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--one-device", "--vectors", "30001", "--steps", "3", "--warmup", "1",
           "--mode", mode, "--no-cpu-baseline", "--dump", str(dump), "--shard-path", path]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, run_fail_msg(r)
    d = np.load(dump, allow_pickle=False)
    codes = d["codes"]
    assert codes.shape == (60002, 8)
    _check_assignment(oracle, d)
    cbs = oracle.build_codebooks(codes, 256, mode == "ctx")
    want, bits = oracle.encode(codes, cbs)
    assert int(d["bits"]) == bits
    assert d["stream"].tobytes() == want


@pytest.mark.parametrize("groups", ["one", "lanes"])
def test_one_rank_rccl_rehearsal_stream(oracle, tmp_path, groups):
    """bench.py --dist-rehearse: the world > 1 pipeline (process group over RCCL, the
    TorchComm hooks, both pqh_shard_encode phases, stream A on its own hardware queue) with
    one rank -- the nccl route on hardware; the rank's stream must equal the oracle's and
    the bench's own checks (round trip, row-path re-encode, shard status) must pass."""
    dump = tmp_path / "dump.npz"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           *_LAUNCH,
           os.path.join(ROOT, "bench.py"), "--dist-rehearse", "--shard-groups", groups,
           "--vectors", "30001", "--steps", "4", "--warmup", "1", "--no-cpu-baseline",
           "--dump", str(dump)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, run_fail_msg(r)
    d = np.load(dump, allow_pickle=False)
    codes = d["codes"]
    assert codes.shape == (30001, 8)
    _check_assignment(oracle, d)
    cbs = oracle.build_codebooks(codes, 256, True)
    want, bits = oracle.encode(codes, cbs)
    assert int(d["bits"]) == bits
    assert d["stream"].tobytes() == want


@pytest.mark.parametrize("config,mode", [("sift", "ctx"), ("deep", "ctx"), ("sift", "noctx")])
def test_one_rank_bench_stream(oracle, tmp_path, config, mode):
    """bench.py exactly as the headline runs it at one rank (no process group: stream A's
    part-major assignment, the histogram and code tables on the table lanes, the part-major
    encoder and the decoder on the encode stream, 4-vector chunks), on a small batch: its last
    batch's codes equal the oracle's assignment and its stream the oracle's encoding of them
    (src/pq_encoder.c:270-272, src/huffman_encoder.c:207-238)."""
    dump = tmp_path / "dump.npz"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--mode", mode,
           "--vectors", "30001", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--device-warmup-ms", "0", "--dump", str(dump)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, run_fail_msg(r)
    d = np.load(dump, allow_pickle=False)
    codes = d["codes"]
    assert codes.shape == (30001, 16 if config == "deep" else 8)
    _check_assignment(oracle, d)
    cbs = oracle.build_codebooks(codes, 256, mode == "ctx")
    want, bits = oracle.encode(codes, cbs)
    assert int(d["bits"]) == bits
    assert d["stream"].tobytes() == want

