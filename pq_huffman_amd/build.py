"""Build libpqh.so and the CLI tools in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m pq_huffman_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs: int = 8) -> str:
    env = dict(os.environ)
    env.setdefault("ARCH", "gfx950")
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "csrc"), f"-j{jobs}"], env=env)
    return os.path.join(HERE, "lib", "libpqh.so")


if __name__ == "__main__":
    print(build(int(sys.argv[1]) if len(sys.argv) > 1 else 8))
