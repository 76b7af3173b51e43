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
