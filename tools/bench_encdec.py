"""Encode / decode alone on the bench's own data (diagnostic): per-launch HIP-event times of
pqh_encode_write_parts (the bench's encoder), pqh_encode_write (row-major) and pqh_decode,
at --rows rows (the batch repeated to fill it), SIFT or Deep shape.

    python tools/bench_encdec.py [--config sift|deep] [--rows 1000000] [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from pq_huffman_amd import codec  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sift")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=4)
    ap.add_argument("--enc-impl", type=int, default=0, help="PQH_TUNE_ENC_IMPL: 1 tiled, 2 one-pass")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    d, m = (128, 8) if a.config == "sift" else (96, 16)
    gen = bench.make_data if a.config == "sift" else bench.make_deep
    base = 1_000_000
    x = gen(torch, base, d, 0x5EED, 0, dev)
    cent = bench.train_centroids(torch, gen(torch, 200_000, d, 0x5EED, 0, dev), m, 256)
    ctx = codec.Context(0)
    ctx.set_tuning(enc_impl=a.enc_impl)
    pq = codec.PQ(ctx, cent)
    rows1 = pq.assign(x)
    del x
    reps = (a.rows + base - 1) // base
    rows = rows1.repeat(reps, 1)[:a.rows].contiguous()
    n = rows.shape[0]
    ld = (n + 127) // 128 * 128
    parts = torch.empty((m, ld), dtype=torch.uint8, device=dev)[:, :n]
    parts.copy_(rows.t())
    counts = codec.histogram(ctx, rows, 256, True)
    tabs = codec.Tables(ctx, m, 256, True).build(counts)
    C = a.chunk
    chunks = (n + C - 1) // C
    out = torch.empty(n * m * 7 + 64, dtype=torch.uint8, device=dev)
    coff = torch.empty(chunks, dtype=torch.int64, device=dev)
    cprev = torch.empty((chunks, m), dtype=torch.uint8, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    t_pm = timed(lambda: codec.encode_write_parts(ctx, tabs, parts, n, out, 0, 1, None, C, coff,
                                                  cprev, total=tot), a.reps)
    t_rw = timed(lambda: codec.encode_write(ctx, tabs, rows, out, 0, 1, None, C, coff, cprev,
                                            total=tot), a.reps)
    codec.encode_status(ctx)
    bits = int(tot.item())
    enc = codec.Encoded(out, bits, C, coff, cprev, n, 1)
    dec = torch.empty_like(rows)
    t_dec = timed(lambda: codec.decode(ctx, tabs, enc, out=dec), a.reps)
    codec.decode_status(ctx)
    assert torch.equal(dec, rows)
    per = 1e6 / n
    print(f"{a.config} impl={a.enc_impl} C={C} rows={n} bits/row={bits / n:.2f}  encode_parts {t_pm * 1e3 * per:.1f} us/1M  "
          f"encode_rows {t_rw * 1e3 * per:.1f} us/1M  decode {t_dec * 1e3 * per:.1f} us/1M", flush=True)


if __name__ == "__main__":
    main()
