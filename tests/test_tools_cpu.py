"""CLI tools that need no GPU: prepend_vecsl_meta (src/prepend_vecsl_meta.c:12-71) against the
reference binary built from its own sources (oracle/ref.mk -> oracle/_ref/), and against the
format itself (u32 N, u32 D, then the payload: src/vecs_io.c:70-76)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

OURS = os.path.join(ROOT, "pq_huffman_amd", "bin", "prepend_vecsl_meta")
REF = os.path.join(ROOT, "oracle", "_ref", "prepend_vecsl_meta")


def _run(exe, path, n, d):
    r = subprocess.run([exe, str(path), str(n), str(d)], capture_output=True, text=True)
    return r.returncode, r.stdout


@pytest.mark.parametrize("kind,dtype", [("b", np.uint8), ("i", np.int32), ("f", np.float32),
                                        ("l", np.int64)])
def test_prepend_vecsl_meta(tmp_path, kind, dtype):
    rng = np.random.default_rng(3)
    n, d = 123, 7
    data = rng.integers(0, 100, (n, d)).astype(dtype)
    want = np.array([n, d], np.uint32).tobytes() + data.tobytes()
    exes = [("ours", OURS)] + ([("ref", REF)] if os.path.exists(REF) else [])
    for name, exe in exes:
        p = tmp_path / f"{name}.{kind}vecsl"
        p.write_bytes(data.tobytes())
        assert _run(exe, p, n, d) == (0, ""), name
        assert p.read_bytes() == want, name
        rc, out = _run(exe, p, n, d)            # already processed: reported, unchanged
        assert (rc, out) == (0, f"File {p} already processed\n"), name
        assert p.read_bytes() == want
        bad = tmp_path / f"{name}_bad.{kind}vecsl"   # wrong size: refused, untouched
        bad.write_bytes(data.tobytes()[:-1])
        assert _run(exe, bad, n, d)[0] == 1, name
        assert bad.read_bytes() == data.tobytes()[:-1]
    missing = tmp_path / "none.fvecsl"
    assert _run(OURS, missing, 1, 1)[0] == 1
    other = tmp_path / "x.qvecsl"
    other.write_bytes(b"")
    assert _run(OURS, other, 0, 0)[0] == 1     # unknown letter


def test_prepend_vecsl_meta_rewrites_in_place(tmp_path):
    """The file is rewritten in place like the reference's (src/prepend_vecsl_meta.c:65-68):
    same inode and mode, a hard link sees the new bytes, a symlink still points at it."""
    data = np.arange(60, dtype=np.float32).tobytes()
    want = np.array([6, 10], np.uint32).tobytes() + data
    p = tmp_path / "x.fvecsl"
    p.write_bytes(data)
    os.chmod(p, 0o640)
    link = tmp_path / "hard.fvecsl"
    os.link(p, link)
    sym = tmp_path / "sym.fvecsl"
    os.symlink(p, sym)
    ino = os.stat(p).st_ino
    assert _run(OURS, sym, 6, 10) == (0, "")
    assert os.path.islink(sym) and sym.read_bytes() == want
    assert os.stat(p).st_ino == ino and (os.stat(p).st_mode & 0o777) == 0o640
    assert link.read_bytes() == want
    assert not any(q.name.endswith(".pqh_tmp") for q in tmp_path.iterdir())
