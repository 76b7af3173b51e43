"""pq_huffman_amd -- MI355X-native PQ + Huffman vector compressor (gfx950).

The product is the C-ABI library pq_huffman_amd/lib/libpqh.so (headers in include/) with
hand-written HIP kernels; this package is its Python mirror (ctypes) used by the tests,
the benchmark and the smoke check.  See DESIGN.md.
"""
from .capi import LIB_PATH, PqhError, lib  # noqa: F401

__all__ = ["lib", "LIB_PATH", "PqhError"]
