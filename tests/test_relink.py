"""INTEGRATION.md section 2 in practice: the reference's own huffman_encoder.c and
huffman_decoder.c (with its mst.c / dsu.c forest loader), compiled against include/*.h and
linked with libpqh instead of the reference's library objects (oracle/ref.mk,
oracle/_ref/relink/), must write the same files as the reference built from its own
sources (oracle/_ref/huffman_encoder, _decoder) -- byte for byte, stdout included.

Build-container only: needs /root/reference (the relinked tools are compiled from its
sources by __graft_entry__.build()); skipped elsewhere.  --no-context is not run: the
shipped encoder reads past a 256-item codebook there (huffman_encoder.c:403-404)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden
import datagen

REF = os.path.join(ROOT, "oracle", "_ref")
RELINK = os.path.join(REF, "relink")

pytestmark = pytest.mark.skipif(
    not (os.path.isdir("/root/reference/src") and os.path.exists(os.path.join(RELINK, "huffman_encoder"))),
    reason="needs the reference sources (build container) and the relinked tools")

FILES = ["huffman_codebooks.bin", "huffman_indices.bin", "huffman_stats.txt"]
TREE_FILES = FILES + ["huffman_children_codebooks.bin", "huffman_children.bin",
                      "huffman_children_stats.txt"]


def _encode(tool_dir, codes, flags, work):
    pq = os.path.join(work, "pq") + "/"
    out = os.path.join(work, "out") + "/"
    os.makedirs(pq, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    datagen.write_vecsl(pq + "pq_indices.bvecsl", codes)
    r = subprocess.run([os.path.join(tool_dir, "huffman_encoder"), pq, out, str(codes.shape[1])]
                       + flags, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return out, r.stdout


def _decode(tool_dir, enc_dir, flags, work):
    outf = os.path.join(work, "decoded.bin")
    r = subprocess.run([os.path.join(tool_dir, "huffman_decoder"), enc_dir, "--output-file", outf]
                       + flags, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return open(outf, "rb").read(), r.stdout


def _inputs():
    yield "m8_n1000", golden("huff_m8_n1000.npz")["input"]
    yield "m16_n1000", golden("huff_m16_n1000.npz")["input"]
    yield "m8_n20000", datagen.skewed_codes(20000, 8, 256, seed=91)


@pytest.mark.parametrize("flags", [[], ["--no-sort"]], ids=["sort_ctx", "nosort_ctx"])
def test_relinked_reference_cli_matches_reference(tmp_path, flags):
    for name, codes in _inputs():
        wa, wb = str(tmp_path / (name + "_ref")), str(tmp_path / (name + "_relink"))
        ea, oa = _encode(REF, codes, flags, wa)
        eb, ob = _encode(RELINK, codes, flags, wb)
        assert oa == ob, name
        for f in FILES:
            assert open(ea + f, "rb").read() == open(eb + f, "rb").read(), (name, f)
        da, _ = _decode(REF, ea, [], wa)
        db, _ = _decode(RELINK, eb, [], wb)
        assert da == db, name


def test_relinked_reference_cli_tree_mode(tmp_path):
    g = golden("huff_tree_m8_n1000.npz")
    tree = str(tmp_path / "mst.tree")
    datagen.write_tree(tree, len(g["counts"]), g["targets"], g["counts"])
    for flags in (["--no-sort", "--tree", tree], ["--tree", tree]):
        wa, wb = str(tmp_path / "ref"), str(tmp_path / "relink")
        ea, oa = _encode(REF, g["input"], flags, wa)
        eb, ob = _encode(RELINK, g["input"], flags, wb)
        assert oa == ob
        for f in TREE_FILES:
            assert open(ea + f, "rb").read() == open(eb + f, "rb").read(), f
        da, _ = _decode(REF, ea, ["--tree"], wa)
        db, _ = _decode(RELINK, eb, ["--tree"], wb)
        assert da == db
        assert np.frombuffer(db, np.uint8).size == g["input"].size
