"""Pin the CPU oracle against outputs of the reference itself (tests/golden/, produced by
oracle/gen_golden.py from /root/reference/src builds) and the reference's embedded
known-answer tests.  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, golden


def _dump(lens, codes, alphabet, context):
    """huffman_codebook_dump format (huffman_codebook.c:6-33)."""
    lines = []
    for i in range(len(lens)):
        head = f"{i // alphabet} -> {i % alphabet}: " if context else f"{i}: "
        if lens[i] == 0:
            lines.append(head + "-")
        else:
            bits = "".join(str((codes[i][b // 8] >> (7 - b % 8)) & 1) for b in range(lens[i]))
            lines.append(head + f"{bits} ({lens[i]})")
    return "\n".join(lines) + "\n"


def test_known_answer_bitstream(oracle):
    ka = json.load(open(os.path.join(GOLD, "known_answers.json")))
    # bitstream.c:196-228: 4 bits of 0x12, 12 bits of 0x34 0x56, 28 bits of 0x78..0xbc
    data = np.array([0x12, 0x34, 0x56, 0x78, 0x9a, 0xbc, 0xde], np.uint8)
    packed = np.concatenate([data[0:1], data[1:3], data[3:7]])
    out = oracle.bitstream_write(packed, [4, 12, 28])
    assert out.hex() == ka["bitstream_test_bytes"] == "1345789abcd0"
    bits = "".join(f"{b:08b}" for b in out)
    assert bits == ka["bitstream_expected_bits"]
    assert ka["bitstream_test_exit"] == 1  # the reference test exits at EOF


def test_known_answer_encode_dump(oracle):
    ka = json.load(open(os.path.join(GOLD, "known_answers.json")))
    t10 = np.array([0, 21, 13, 8, 5, 3, 2, 1, 1, 0], float)
    text = ""
    for context, nz in ((0, -1), (0, 1), (0, 0), (1, -1)):   # huffman_encode.c:315-318
        c = np.zeros(100)
        c[:10] = t10
        if 0 <= nz < 3:
            c[nz + 1:10] = 0
        if context:
            for i in range(10, 100):
                c[i] = c[i - 10 + 1]
            lens, codes = oracle.codebook(10, c, context=True)
        else:
            lens, codes = oracle.codebook(10, c[:10])
        text += _dump(lens, codes, 10, context)
    assert text == ka["huffman_encode_test_dump"]


def test_known_answer_decode(oracle):
    """huffman_decode.c:196-221: codebook from {1,4,3,8,3,8}; round trip of the string."""
    ka = json.load(open(os.path.join(GOLD, "known_answers.json")))
    assert "abacabadabacabaeabacabadabacaba" in ka["huffman_decode_test_stdout"]
    lens, codes = oracle.codebook(6, np.array([1.0, 4, 3, 8, 3, 8]))
    cbs = oracle.Codebooks(6, False, lens[None], codes[None], codes.shape[1])
    seq = np.array([0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3,
                    0, 1, 0, 2, 0, 1, 0], np.uint8)[:, None]
    stream, _ = oracle.encode(seq, cbs)
    dec = oracle.decode(stream, len(seq), 1, cbs)
    assert "".join(chr(97 + s) for s in dec[:, 0]) == "abacabadabacabaeabacabadabacaba"


@pytest.mark.parametrize("case", ["fib1024", "fib32ctx", "enc_test_many", "enc_test_one",
                                  "enc_test_zero", "ties_small_ints", "ties_all_equal",
                                  "ties_powers", "single_symbol", "empty", "geometric",
                                  "ctx16_mixed"])
def test_codebook_vs_reference(oracle, case):
    g = golden("codebooks.npz")
    k, c = g[case + "__alphabet"]
    counts = g[case + "__counts"]
    rlens, rcodes = g[case + "__lens"], g[case + "__codes"]
    lens, codes = oracle.codebook(int(k), counts, context=bool(c), stride=rcodes.shape[1])
    assert np.array_equal(lens, rlens)
    assert np.array_equal(codes, rcodes)
    assert oracle.serialize(int(k), bool(c), lens, codes) == g[case + "__file"].tobytes()


@pytest.mark.parametrize("buf", [2, 3, 64])
def test_bitstream_vs_reference(oracle, buf):
    g = golden("bitstream.npz")
    out = oracle.bitstream_write(g[f"buf{buf}__data"], g[f"buf{buf}__lens"])
    assert out == g[f"buf{buf}__out"].tobytes()


MODES = {"sort_ctx": (True, True), "nosort_ctx": (False, True), "nosort_noctx": (False, False)}


@pytest.mark.parametrize("name", ["m8_n1000", "m16_n1000", "m8_n1", "m3_n2"])
@pytest.mark.parametrize("mode", list(MODES))
def test_huffman_files_vs_reference(oracle, name, mode):
    g = golden(f"huff_{name}.npz")
    sort, ctx = MODES[mode]
    codes = g["input"]
    if sort:
        codes = oracle.sort_rows(codes)
    cbs = oracle.build_codebooks(codes, 256, ctx)
    assert oracle.codebooks_file(cbs) == g[mode + "__codebooks"].tobytes()
    assert oracle.indices_file(codes, cbs) == g[mode + "__indices"].tobytes()
    counts = oracle.histogram(codes, 256, ctx)
    stats = oracle.stats_json(len(codes), codes.shape[1], 256, 1 if ctx else 0,
                              oracle.estimate_parts(cbs, counts))
    assert stats == g[mode + "__stats"].tobytes().decode()
    dec = oracle.decode(g[mode + "__indices"].tobytes()[8:], len(codes), codes.shape[1], cbs)
    assert np.array_equal(dec, g[mode + "__decoded"])
    assert np.array_equal(dec, codes)


def test_huffman_n10000_sha(oracle):
    summ = json.load(open(os.path.join(GOLD, "huff_summaries.json")))["m8_n10000"]
    g = golden("huff_m8_n10000.npz")
    for mode, (sort, ctx) in MODES.items():
        codes = oracle.sort_rows(g["input"]) if sort else g["input"]
        cbs = oracle.build_codebooks(codes, 256, ctx)
        assert hashlib.sha256(oracle.codebooks_file(cbs)).hexdigest() == summ[mode]["codebooks_sha256"]
        assert hashlib.sha256(oracle.indices_file(codes, cbs)).hexdigest() == summ[mode]["indices_sha256"]


def test_k4096_noctx_vs_reference(oracle):
    g = golden("huff_k4096_m8_n2000.npz")
    codes = g["input"]
    cbs = oracle.build_codebooks(codes, 4096, False, stride=16)
    assert oracle.codebooks_file(cbs) == g["nosort_noctx__codebooks"].tobytes()
    assert oracle.indices_file(codes, cbs) == g["nosort_noctx__indices"].tobytes()
    dec = oracle.decode(g["nosort_noctx__indices"].tobytes()[8:], len(codes), 8, cbs)
    assert np.array_equal(dec, codes)


def test_sort_is_strncmp_stable(oracle):
    """Sort-mode key: stable sort of rows with bytes after the first 0
    zeroed -- checked against the reference's sorted output encoded in the fixture."""
    g = golden("huff_m8_n1000.npz")
    codes = g["input"]
    s = oracle.sort_rows(codes)
    key = codes.copy()
    for r in key:
        z = np.nonzero(r == 0)[0]
        if len(z):
            r[z[0]:] = 0
    order = np.lexsort(key.T[::-1])  # lexsort is stable
    assert np.array_equal(s, codes[order])
    assert np.array_equal(s, g["sort_ctx__decoded"])


@pytest.mark.parametrize("name", ["sift_n1000_m8_k256", "deep_n500_m16_k256"])
def test_pq_assign_selfconsistent(oracle, name):
    """PQ fixture is self-generated (parity unpinned at the yael boundary): the oracle
    must reproduce it, and each code must be a first minimum of an fp64 re-check within
    the 1e-5 relative distance criterion."""
    g = golden(f"pq_{name}.npz")
    codes, dists = oracle.pq_assign(g["x"], g["centroids"])
    assert np.array_equal(codes, g["codes"])
    assert np.array_equal(dists, g["dists"])
    x, c = g["x"].astype(np.float64), g["centroids"].astype(np.float64)
    m, k, ds = c.shape
    for j in range(m):
        sub = x[:, j * ds:(j + 1) * ds]
        d = ((sub[:, None, :] - c[j][None]) ** 2).sum(-1)
        best = d.min(1)
        chosen = d[np.arange(len(x)), codes[:, j]]
        assert np.all(chosen <= best * (1 + 1e-5) + 1e-12)
