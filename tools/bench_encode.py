"""One-pass encode micro-benchmark with phase stamps of the mid-grid workgroup (diagnostic)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402
from pq_huffman_amd.capi import lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, m, k = 1_000_000, 8, 256
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    base = torch.randint(0, k, (n, m), generator=g, device=dev)
    skew = (torch.rand((n, m), generator=g, device=dev) ** 3 * k).long()
    codes = ((base // 16) * 16 + skew % 16).clamp(0, k - 1).to(torch.uint8)
    ctx = codec.Context(0)
    L = lib()
    L.pqh_debug_enc_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for mode in (True, False):
        items = k * k if mode else k
        counts = torch.zeros((m, items), dtype=torch.int32, device=dev)
        codec.histogram(ctx, codes, k, mode, counts=counts)
        tabs = codec.Tables(ctx, m, k, mode)
        tabs.build(counts)
        out = torch.empty(n * m * 56 // 8 + 64, dtype=torch.uint8, device=dev)
        C = 16
        chunks = (n + C - 1) // C
        coff = torch.empty(chunks, dtype=torch.int64, device=dev)
        cprev = torch.empty((chunks, m), dtype=torch.uint8, device=dev) if mode else None
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        for _ in range(3):
            codec.encode_write(ctx, tabs, codes, out, 0, 1, None, C, coff, cprev, total=tot)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            codec.encode_write(ctx, tabs, codes, out, 0, 1, None, C, coff, cprev, total=tot)
        e1.record()
        torch.cuda.synchronize()
        st = (ctypes.c_ulonglong * 8)()
        L.pqh_debug_enc_stamps(ctx.ptr, st)
        st = list(st)
        print(f"ctx={mode} encode_ms={e0.elapsed_time(e1) / 10:.4f} mid-wg cycles: "
              f"gather={st[1]-st[0]} lookback={st[2]-st[1]} image={st[3]-st[2]} "
              f"tail={st[4]-st[3]} store={st[5]-st[4]} start_offset_from_first? bits={int(tot.item())}",
              flush=True)


if __name__ == "__main__":
    main()
