#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

Runs in the build container only (it needs /root/reference).  Every expected output here
is produced by the REFERENCE ITSELF, compiled from /root/reference/src by oracle/ref.mk
into oracle/_ref/ -- the CLI binaries (huffman_encoder, huffman_decoder) as shipped, the
embedded _X_TEST mains, and libref.so (reference library + oracle/ref_harness.c driver
for the two cases the shipped CLI cannot run: --no-context and K=4096).

The only self-generated fixture is pq_*.npz: PQ assignment parity is unpinned at the yael
boundary (yael v438 absent), so its expected codes come from the oracle's documented
definition (oracle/pqh_oracle.c header) and are labelled as such.

    python oracle/gen_golden.py
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.join(ROOT, "tests", "golden")


def build():
    subprocess.check_call(["make", "-s", "-f", "oracle/ref.mk", "-j8"], cwd=ROOT)
    subprocess.check_call(["make", "-s", "-f", "oracle/Makefile"], cwd=ROOT)


def reflib():
    lib = ctypes.CDLL(os.path.join(REF, "libref.so"))
    P, I, LL, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_char_p
    lib.refh_build_codebook.argtypes = [I, I, P, P, P, I]
    lib.refh_save_codebook_file.argtypes = [I, I, P, D]
    lib.refh_encode_dir.argtypes = [D, P, I, LL, I, I, I]
    lib.refh_decode_dir.argtypes = [D, P, I, LL]
    lib.refh_bitstream_write.argtypes = [D, P, P, I, LL]
    return lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def read(p):
    with open(p, "rb") as f:
        return f.read()


def known_answers(tmp):
    out = {}
    # bitstream.c:196-228 writes 4+12+28 bits through a 2-byte buffer to /tmp/foo.bin and
    # exits 1 at EOF before its assert -- the bytes are the answer.
    r = subprocess.run([os.path.join(REF, "bitstream_test")], cwd=tmp, capture_output=True)
    out["bitstream_test_exit"] = r.returncode
    out["bitstream_test_bytes"] = read("/tmp/foo.bin").hex()
    out["bitstream_expected_bits"] = "000100110100010101111000100110101011110011010000"
    r = subprocess.run([os.path.join(REF, "huffman_encode_test"), "-v"], capture_output=True,
                       text=True, check=True)
    out["huffman_encode_test_dump"] = r.stdout
    r = subprocess.run([os.path.join(REF, "huffman_decode_test")], capture_output=True,
                       text=True, check=True)
    out["huffman_decode_test_stdout"] = r.stdout
    r = subprocess.run([os.path.join(REF, "huffman_codebook_test")], capture_output=True,
                       text=True, check=True)
    out["huffman_codebook_test_stdout"] = r.stdout
    out["huffman_codebook_test_last_file_sha256"] = hashlib.sha256(
        read("/tmp/codebook.bin")).hexdigest()
    with open(os.path.join(GOLD, "known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)


def codebook_fixtures(lib, tmp):
    """Reference codebooks (lengths, codes, serialised file) for count tables that stress
    the heap tie-breaks (huffman_encode.c:33-76) and the 0/1-symbol special cases."""
    cases = {}
    fib = np.zeros(1024)
    fib[1] = 1.0
    for i in range(2, 1024):
        fib[i] = fib[i - 1] + fib[i - 2]
    cases["fib1024"] = (1024, 0, fib)                       # huffman_codebook.c:148-165
    fibc = np.zeros(32 * 32)
    fibc[1] = 1.0
    for i in range(2, 1024):
        fibc[i] = fibc[i - 1] + fibc[i - 2]
    cases["fib32ctx"] = (32, 1, fibc)
    t10 = np.array([0, 21, 13, 8, 5, 3, 2, 1, 1, 0], float)  # huffman_encode.c:284
    cases["enc_test_many"] = (10, 0, t10)
    cases["enc_test_one"] = (10, 0, np.where(np.arange(10) <= 1, t10, 0))
    cases["enc_test_zero"] = (10, 0, np.where(np.arange(10) <= 0, t10, 0))
    rng = np.random.default_rng(3)
    cases["ties_small_ints"] = (256, 0, rng.integers(0, 4, 256).astype(float))
    cases["ties_all_equal"] = (256, 0, np.ones(256))
    cases["ties_powers"] = (64, 0, np.array([2.0 ** (i % 7) for i in range(64)]))
    cases["single_symbol"] = (256, 0, np.eye(256)[17] * 5)
    cases["empty"] = (256, 0, np.zeros(256))
    cases["geometric"] = (256, 0, np.bincount(np.minimum(rng.geometric(0.03, 20000) - 1, 255),
                                               minlength=256).astype(float))
    ctx = rng.integers(0, 3, (16, 16)).astype(float)
    ctx[3] = 0.0
    ctx[5] = 0.0
    ctx[5, 9] = 4.0
    cases["ctx16_mixed"] = (16, 1, ctx.ravel())
    arrays = {}
    for name, (k, c, counts) in cases.items():
        counts = np.ascontiguousarray(counts, np.float64)
        items = k * k if c else k
        stride = (k + 7) // 8 + 1
        lens = np.zeros(items, np.int32)
        codes = np.zeros((items, stride), np.uint8)
        rc = lib.refh_build_codebook(k, c, ptr(counts), ptr(lens), ptr(codes), stride)
        assert rc == 0, name
        path = os.path.join(tmp, name + ".cb")
        assert lib.refh_save_codebook_file(k, c, ptr(counts), path.encode()) == 0
        arrays[name + "__alphabet"] = np.array([k, c])
        arrays[name + "__counts"] = counts
        arrays[name + "__lens"] = lens
        arrays[name + "__codes"] = codes
        arrays[name + "__file"] = np.frombuffer(read(path), np.uint8)
    np.savez_compressed(os.path.join(GOLD, "codebooks.npz"), **arrays)


def run_cli_encode(codes, flags, tmp, tag):
    pq = os.path.join(tmp, tag + "_pq") + "/"
    out = os.path.join(tmp, tag + "_out") + "/"
    os.makedirs(pq, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    datagen.write_vecsl(pq + "pq_indices.bvecsl", codes)
    m = codes.shape[1]
    r = subprocess.run([os.path.join(REF, "huffman_encoder"), pq, out, str(m)] + flags,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out, r.stdout


def run_cli_decode(enc_dir, n, m, tmp, tag):
    outf = os.path.join(tmp, tag + "_decoded.bin")
    r = subprocess.run([os.path.join(REF, "huffman_decoder"), enc_dir, "--output-file", outf],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return np.fromfile(outf, np.uint8).reshape(n, m)


def huffman_mode_fixtures(lib, tmp, n, m, seed, name, full=True):
    codes = datagen.skewed_codes(n, m, 256, seed=seed)
    arrays = {"input": codes}
    summary = {}
    for mode, flags in (("sort_ctx", []), ("nosort_ctx", ["--no-sort"]),
                        ("nosort_noctx", None)):
        tag = f"{name}_{mode}"
        if flags is None:
            # --no-context as shipped reads past a 256-item codebook (huffman_encoder.c:403);
            # run the same flow through the reference library (oracle/ref_harness.c).
            out = os.path.join(tmp, tag + "_out") + "/"
            os.makedirs(out, exist_ok=True)
            c = np.ascontiguousarray(codes)
            assert lib.refh_encode_dir(out.encode(), ptr(c), 1, n, m, 256, 0) == 0
            stdout = ""
        else:
            out, stdout = run_cli_encode(codes, flags, tmp, tag)
        dec = run_cli_decode(out, n, m, tmp, tag)
        cb = read(out + "huffman_codebooks.bin")
        ix = read(out + "huffman_indices.bin")
        st = read(out + "huffman_stats.txt").decode()
        summary[mode] = {"codebooks_sha256": hashlib.sha256(cb).hexdigest(),
                         "codebooks_size": len(cb),
                         "indices_sha256": hashlib.sha256(ix).hexdigest(),
                         "indices_size": len(ix), "stats": st,
                         "decoded_sha256": hashlib.sha256(dec.tobytes()).hexdigest()}
        if full:
            arrays[mode + "__codebooks"] = np.frombuffer(cb, np.uint8)
            arrays[mode + "__indices"] = np.frombuffer(ix, np.uint8)
            arrays[mode + "__stats"] = np.frombuffer(st.encode(), np.uint8)
            arrays[mode + "__decoded"] = dec
    np.savez_compressed(os.path.join(GOLD, f"huff_{name}.npz"), **arrays)
    return summary


def tree_fixtures(tmp, n=1000, m=8, seed=21, roots=3, name="tree_m8_n1000"):
    """Tree mode (huffman_encoder --tree mst.tree, huffman_decoder --tree) on a seeded
    forest in the reference's mst.tree layout, with and without the default sort."""
    codes = datagen.skewed_codes(n, m, 256, seed=seed)
    targets, counts = datagen.random_forest(n, roots=roots, seed=seed)
    tree = os.path.join(tmp, name + ".tree")
    datagen.write_tree(tree, n, targets, counts)
    arrays = {"input": codes, "targets": targets, "counts": counts}
    for mode, flags in (("tree_nosort", ["--no-sort"]), ("tree_sort", [])):
        out, _ = run_cli_encode(codes, flags + ["--tree", tree], tmp, f"{name}_{mode}")
        outf = os.path.join(tmp, f"{name}_{mode}_decoded.bin")
        r = subprocess.run([os.path.join(REF, "huffman_decoder"), out, "--output-file", outf,
                            "--tree"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        arrays[mode + "__decoded"] = np.fromfile(outf, np.uint8).reshape(n, m)
        for f in ("huffman_codebooks.bin", "huffman_indices.bin",
                  "huffman_children_codebooks.bin", "huffman_children.bin",
                  "huffman_stats.txt", "huffman_children_stats.txt"):
            arrays[mode + "__" + f.split(".")[0]] = np.frombuffer(read(out + f), np.uint8)
    np.savez_compressed(os.path.join(GOLD, f"huff_{name}.npz"), **arrays)


def k4096_fixture(lib, tmp):
    n, m = 2000, 8
    codes = datagen.skewed_codes(n, m, 4096, seed=11, p=0.004)
    out = os.path.join(tmp, "k4096_out") + "/"
    os.makedirs(out, exist_ok=True)
    c = np.ascontiguousarray(codes)
    assert lib.refh_encode_dir(out.encode(), ptr(c), 2, n, m, 4096, 0) == 0
    dec = np.zeros_like(c)
    assert lib.refh_decode_dir(out.encode(), ptr(dec), 2, n) == 0
    assert np.array_equal(dec, c)
    np.savez_compressed(os.path.join(GOLD, "huff_k4096_m8_n2000.npz"), input=codes,
                        nosort_noctx__codebooks=np.frombuffer(read(out + "huffman_codebooks.bin"), np.uint8),
                        nosort_noctx__indices=np.frombuffer(read(out + "huffman_indices.bin"), np.uint8),
                        nosort_noctx__stats=np.frombuffer(read(out + "huffman_stats.txt"), np.uint8))


def bitstream_fixture(lib, tmp):
    """Reference writer with tiny buffers (mid-stream flush path) on random writes."""
    rng = np.random.default_rng(5)
    arrays = {}
    for buf in (2, 3, 64):  # 1-byte buffers loop forever in the reference (bitstream.c:131-147)
        lens = rng.integers(0, 40, 300).astype(np.int64)
        data = b"".join(bytes(rng.integers(0, 256, (int(L) + 7) // 8, dtype=np.uint8)) for L in lens)
        dbuf = np.frombuffer(data, np.uint8).copy()
        path = os.path.join(tmp, f"bs{buf}.bin")
        assert lib.refh_bitstream_write(path.encode(), ptr(dbuf), ptr(lens), len(lens), buf) == 0
        arrays[f"buf{buf}__lens"] = lens
        arrays[f"buf{buf}__data"] = dbuf
        arrays[f"buf{buf}__out"] = np.frombuffer(read(path), np.uint8)
    np.savez_compressed(os.path.join(GOLD, "bitstream.npz"), **arrays)


def pq_fixtures():
    """SELF-GENERATED (parity unpinned at the yael boundary): seeded inputs, fixed
    centroids, and the oracle's codes + fp32 distances."""
    orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "liboracle.so"))
    orc.orc_pq_assign.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_int]
    for name, x, m, k in (("sift_n1000_m8_k256", datagen.sift_like(1000), 8, 256),
                          ("deep_n500_m16_k256", datagen.deep_like(500), 16, 256)):
        cent = datagen.lloyd_centroids(x, m, k, iters=3, sample=len(x))
        codes = np.zeros((len(x), m), np.uint8)
        dists = np.zeros((len(x), m), np.float32)
        orc.orc_pq_assign(ptr(x), len(x), x.shape[1], m, k, ptr(cent), ptr(codes), 1,
                          ptr(dists), 1)
        np.savez_compressed(os.path.join(GOLD, f"pq_{name}.npz"), x=x, centroids=cent,
                            codes=codes, dists=dists, note=np.frombuffer(
                                b"self-generated: oracle definition, parity unpinned (yael absent)",
                                np.uint8))


def forest_fixtures(tmp):
    """The forest builder: the REFERENCE's block geometry (blocks_info_init over an .fvecs,
    oracle/_ref/libref_knn.so), its block membership (is_vector_in_block), its heap merge
    (fast_nn_heap_push/_sort) of the in-block neighbour lists, and mst_builder's mst.tree
    (oracle/_ref/mst_builder) for three take / penalty settings.  The in-block neighbour
    lists themselves (yael's knn_full_thread in the reference) are SELF-GENERATED by the
    oracle's definition -- parity unpinned at that call -- and stored as the push log."""
    sys.path.insert(0, ROOT)
    from oracle import oracle_ctypes as oc
    R = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_knn.so"))
    P = ctypes.c_void_p
    R.refk_blocks_info.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_double, P, P]
    R.refk_in_block.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P,
                                ctypes.c_longlong]
    R.refk_merge.argtypes = [ctypes.c_longlong, ctypes.c_int, ctypes.c_longlong, P, P, P, P, P]
    cases = (("sift_n1200_d16", datagen.sift_like(1200, 16, seed=31), 3, 4, 0.1, 10),
             ("deep_n800_d12", datagen.deep_like(800, 12, seed=32), 2, 5, 0.3, 8))
    for name, x, ns, nb, ov, nn in cases:
        x = np.ascontiguousarray(x, np.float32)
        n, d = x.shape
        fv = os.path.join(tmp, f"{name}.fvecs")
        datagen.write_fvecs(fv, x)
        st = np.zeros((ns, nb), np.float32)
        en = np.zeros_like(st)
        R.refk_blocks_info(fv.encode(), n, d, ns, nb, ov, ptr(st), ptr(en))
        member = np.zeros((nb ** ns, n), np.uint8)
        for b in range(nb ** ns):
            for v in range(n):
                member[b, v] = R.refk_in_block(ptr(x[v]), d, ns, nb, ptr(st), ptr(en), b)
        _, _, sizes, (lr, li, ld) = oc.knn_fast(x, nn, st, en, log=True)
        ri = np.zeros((n, nn), np.uint32)
        rd = np.zeros((n, nn), np.float32)
        R.refk_merge(n, nn, len(lr), ptr(lr), ptr(li), ptr(ld), ptr(ri), ptr(rd))
        nd = os.path.join(tmp, name + "_nn") + "/"
        os.makedirs(nd, exist_ok=True)
        for fn, a in (("nn_indices.ivecsl", ri), ("nn_dist.fvecsl", rd)):
            with open(nd + fn, "wb") as f:
                f.write(np.array([n, nn], np.uint32).tobytes() + a.tobytes())
        codes = datagen.skewed_codes(n, 8, seed=33)
        pqd = os.path.join(tmp, name + "_pq") + "/"
        os.makedirs(pqd, exist_ok=True)
        datagen.write_vecsl(pqd + "pq_indices.bvecsl", codes)
        arrays = dict(x=x, num_split=ns, blocks_per_dim=nb, overlap=ov, num_nn=nn, starts=st,
                      ends=en, member=member, push_row=lr, push_idx=li, push_dist=ld,
                      nn_idx=ri, nn_dist=rd, pq=codes)
        for tag, take, pen in (("t5_p0", 5, "0"), ("t3_p2.5", 3, "2.5"), ("tall_pinf", nn, "inf")):
            od = os.path.join(tmp, f"{name}_{tag}") + "/"
            os.makedirs(od, exist_ok=True)
            subprocess.run([os.path.join(ROOT, "oracle", "_ref", "mst_builder"), nd, od, str(take),
                            "--pq-template", pqd, "--pq-penalty", pen], check=True,
                           capture_output=True)
            arrays[f"tree_{tag}"] = np.frombuffer(read(od + "mst.tree"), np.uint8)
            arrays[f"stats_{tag}"] = np.frombuffer(read(od + "stats.json"), np.uint8)
            arrays[f"stats_children_{tag}"] = np.frombuffer(read(od + "stats_num_children.json"),
                                                            np.uint8)
        np.savez_compressed(os.path.join(GOLD, f"forest_{name}.npz"), **arrays)


def main():
    build()
    if sys.argv[1:] == ["forest"]:   # only the forest-builder fixtures
        tmp = tempfile.mkdtemp(prefix="pqh_golden_")
        try:
            forest_fixtures(tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    if sys.argv[1:] == ["tree"]:   # only the tree-mode fixtures
        tmp = tempfile.mkdtemp(prefix="pqh_golden_")
        try:
            tree_fixtures(tmp)
            tree_fixtures(tmp, n=300, m=16, seed=22, roots=1, name="tree_m16_n300")
            tree_fixtures(tmp, n=64, m=8, seed=23, roots=16, name="tree_m8_n64_forest")
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    os.makedirs(GOLD, exist_ok=True)
    lib = reflib()
    tmp = tempfile.mkdtemp(prefix="pqh_golden_")
    try:
        known_answers(tmp)
        codebook_fixtures(lib, tmp)
        bitstream_fixture(lib, tmp)
        summaries = {}
        summaries["m8_n1000"] = huffman_mode_fixtures(lib, tmp, 1000, 8, 1, "m8_n1000")
        summaries["m16_n1000"] = huffman_mode_fixtures(lib, tmp, 1000, 16, 2, "m16_n1000")
        summaries["m8_n1"] = huffman_mode_fixtures(lib, tmp, 1, 8, 3, "m8_n1")
        summaries["m3_n2"] = huffman_mode_fixtures(lib, tmp, 2, 3, 4, "m3_n2")
        summaries["m8_n10000"] = huffman_mode_fixtures(lib, tmp, 10000, 8, 5, "m8_n10000",
                                                       full=False)
        with open(os.path.join(GOLD, "huff_summaries.json"), "w") as f:
            json.dump(summaries, f, indent=1)
        k4096_fixture(lib, tmp)
        pq_fixtures()
        forest_fixtures(tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print("golden fixtures written to", GOLD)


if __name__ == "__main__":
    main()
