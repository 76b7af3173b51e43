#!/usr/bin/env python3
"""Benchmark: encode+decode round trip of the PQ+Huffman hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode ctx|noctx]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Workload (BASELINE.json configs[1], SIFT1M-shaped): per GPU 1,000,000 synthetic SIFT-like
128-d fp32 vectors resident in HBM, M=8 sub-spaces, K=256 centroids (weak scaling: every
rank owns its own 1M-vector shard).  One step = the reference pipeline
pq_encoder (assignment) -> huffman_encoder -> huffman_decoder on device-resident data:

    pq_assign (MFMA screen + exact re-rank) -> symbol histogram [-> RCCL all-reduce]
    -> GPU codebooks (reference heap tie-breaks) + decode tables -> encode size
    [-> all-gather of shard bit totals and halo rows] -> encode write -> chunked decode

value = vectors round-tripped by all ranks / wall time (Mvec/s).  `roofline` is for the
dominant kernel, pq_assign: algorithmic bytes = 512 B read per vector (+8 B codes) over
its HIP-event-timed duration against 8 TB/s HBM.  `cpu_baseline` times the CPU oracle
(a byte-exact restatement of the reference, tests/test_oracle_golden.py) on a bounded
sample on this host, rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mvec/s encode+decode round-trip, 128-d fp32 M=8 K=256; % HBM-read roofline"
HBM_PEAK_GBS = 8000.0
BYTES_PER_VEC_READ = 512          # 128 fp32
BYTES_PER_VEC_WRITE = 8           # M=8 uint8 codes
ROOT = os.path.dirname(os.path.abspath(__file__))


# the assignment kernel instantiation each configuration runs (its rocprof short name)
ASSIGN_KERNEL = {"sift": "pq_assign_mfma<16, 8, unsigned char>",
                 "deep": "pq_assign_mfma<6, 8, unsigned char>",
                 "k4096": "pq_assign_mfma<16, 128, unsigned short>"}


def profile_tag(config, sort, vectors=1_000_000):
    """the profiles/ tag of a bench configuration (profiles/collect.sh r<N>_<tag>): sift,
    deep, k4096, sift_sort; another batch size adds its millions (sift at 125M rows: 125m,
    collected by profiles/collect.sh r<N>_125m --vectors 125000000 ...)"""
    tag = config + ("_sort" if sort else "")
    if vectors != 1_000_000:
        tag = f"{vectors // 1_000_000}m" if tag == "sift" else f"{tag}_{vectors // 1_000_000}m"
    return tag


def pmc_traffic(kernel, tag):
    """HBM bytes per launch and the kernel-trace average of exactly `kernel` (the
    instantiation this configuration runs) from the newest committed profile of THIS
    configuration: profiles/r<N>_<tag>_pmc_summary.json, written by profiles/summarize.py
    from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench command."""
    import glob
    import re
    files = []
    for f in glob.glob(os.path.join(ROOT, "profiles", f"r*_{tag}_pmc_summary.json")):
        # r<N>_<tag> or r<N>_final_<tag> (a round's last profile of the configuration)
        mt = re.match(r"r(\d+)_(final_)?" + re.escape(tag) + r"_pmc_summary\.json$",
                      os.path.basename(f))
        if mt:
            files.append((int(mt.group(1)), 1 if mt.group(2) else 0, f))
    for *_, f in sorted(files, reverse=True):
        try:
            e = json.load(open(f))["kernels"].get(kernel)
        except (OSError, ValueError, KeyError):
            continue
        if e and "hbm_bytes" in e:
            return e["hbm_bytes"], os.path.relpath(f, ROOT), e.get("avg_us")
    return None, None, None


def lib_shard_req(args, multi):
    """world > 1 (or --dist-rehearse) through the C ABI's two-phase shard encode (bench's
    default there)"""
    return multi and args.shard_path == "library" and not args.sort and \
        not (args.sched == "serial" or args.no_overlap)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 steps = 200 M vectors, ~0.1 s: the lanes pipeline fills and drains inside the timed
    # region, and at 30 steps that costs ~7 % of the steady-state rate
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--vectors", type=int, default=1_000_000, help="vectors per GPU")
    ap.add_argument("--mode", choices=["ctx", "noctx"], default="ctx")
    ap.add_argument("--config", choices=["sift", "deep", "k4096"], default="sift",
                    help="sift: BASELINE configs[1]/[2] (128-d, M=8, K=256; the headline); "
                         "deep: configs[3] (96-d unit-norm, M=16, K=256); k4096: configs[4] "
                         "(128-d, M=8, K=4096, u16 codes, non-context)")
    ap.add_argument("--sort", action="store_true",
                    help="the reference's default mode: rows sorted by the strncmp key before "
                         "the context histogram and encode (huffman_encoder.c:301-318); the "
                         "round trip then returns the sorted rows")
    ap.add_argument("--chunk", type=int, default=4,
                    help="vectors per decode chunk (chunk-index granularity: the encoder writes "
                         "each chunk's bit offset (8 B) and context row (m B) beside the stream, "
                         "and the decoder runs one lookup chain per chunk -- the decode is bound "
                         "by that chain's latency, so more, shorter chains decode faster: chunk "
                         "4 vs 8 measured 45 vs 58 us alone per 1M SIFT rows, 141 vs 247 Deep; "
                         "bench 2,976-3,008 vs 2,856-2,858 Mvec/s, Deep 1,538 vs 1,356)")
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sched", choices=["lanes", "serial"], default="lanes",
                    help="'lanes': assignment + histogram on one stream, each batch's code "
                         "tables, encode and decode on one of --lanes streams (overlapped); "
                         "'serial': every stage in order on one stream")
    ap.add_argument("--no-overlap", action="store_true", help="same as --sched serial")
    ap.add_argument("--lanes", type=int, default=None,
                    help="streams taking batches round robin for tables + encode + decode "
                         "(default 2; 3 for --config k4096, whose tree builds are the long "
                         "stage: 230 vs 219 Mvec/s)")
    ap.add_argument("--elanes", type=int, default=None,
                    help="> 0: encode + decode on this many streams of their own; the --lanes "
                         "streams then build code tables only (default 1; 0 for k4096)")
    ap.add_argument("--drain-trees", choices=["default", "grp", "wave", "lane"],
                    default="default",
                    help="tree builder of the run's last batch, built after the assignment "
                         "stream is done (default: the library's, 16 lanes per tree for "
                         "k <= 256)")
    ap.add_argument("--fill-trees", choices=["default", "grp", "wave", "lane"],
                    default="default",
                    help="tree builder of the first batch on each table lane (the pipeline's "
                         "fill)")
    ap.add_argument("--device-warmup-ms", type=float, default=100.0,
                    help="untimed setup before the warmup steps: the assignment kernel alone for "
                         "this long, so the timed steps run at the GPU's sustained clocks")
    ap.add_argument("--hist-split", choices=["on", "off"], default="on",
                    help="context histogram in two halves: the per-chunk partial counts on the "
                         "assignment stream, their reduce on the batch's table lane")
    ap.add_argument("--stage-events", choices=["after", "timed"], default="after",
                    help="per-stage HIP events other than the assignment's: recorded in extra "
                         "untimed steps after the timed region (default: an event record is a "
                         "packet on its stream, +2-3 %% when all ride in the timed steps), or "
                         "inside the timed steps; the assignment's (the roofline kernel) are "
                         "always recorded in the timed steps")
    ap.add_argument("--encode-after", choices=["tables", "trees"], default="tables",
                    help="the encode waits for the batch's whole tables, or (trees) only for its "
                         "Huffman trees when they completed the encode tables (group builder), "
                         "running beside the decode-table build")
    ap.add_argument("--astreams", type=int, default=1,
                    help="assignment + histogram streams, batch i on stream i %% N (N > 1: the "
                         "next batch's assignment grid fills the previous one's tail)")
    ap.add_argument("--code-layout", choices=["rows", "parts"], default="parts",
                    help="parts (default where it applies: one rank, no sort, u8 codes, m = 8 "
                         "or 16): the assignment writes part-major codes (whole lines) that the "
                         "histogram and the row encoder read directly; rows: pq_indices.bvecsl "
                         "order (measured: parts 2,572-2,673 vs rows 2,481-2,544 Mvec/s at 1M, "
                         "3,273 vs 3,135 at the 125M-row shard)")
    ap.add_argument("--sort-on", choices=["assign", "lanes"], default="lanes",
                    help="--sort: the sort (and then the histogram) of batch i on its table lane "
                         "after its assignment (default), or on the assignment stream")
    ap.add_argument("--hist-on", choices=["auto", "assign", "lanes", "own"], default="auto",
                    help="stream of the context histogram: the assignment's, the batch's "
                         "lane (before its code tables; --hist-tune shapes it to fit beside the "
                         "assignment grid), or a stream of its own (a fifth stream: the process "
                         "then asks HIP for 8 hardware queues); auto: lanes below 16M rows per "
                         "batch, else the assignment's (measured: 1M rows 3,118-3,127 vs "
                         "3,000-3,009 Mvec/s at 200 steps, Deep 1,554-1,569 vs 1,530-1,535; "
                         "125M rows 3,633 vs 3,674)"),
    ap.add_argument("--assign-event-every", type=int, default=4,
                    help="record the assignment's start/end HIP events (the roofline's kernel "
                         "time) on every N-th timed step (0: none -- the roofline then uses the "
                         "untimed steps after the timed region).  An event record is a packet "
                         "on stream A: every step 2,531-2,550 Mvec/s, every 4th 2,575-2,604, "
                         "none 2,599-2,613 (200 steps)")
    ap.add_argument("--assign-wgs-per-cu", type=float, default=2.5,
                    help="workgroups per CU of the persistent K = 256 assignment grid "
                         "(PQH_ASSIGN_WGS_PER_CU; the occupancy limit is 3): with three 166-VGPR "
                         "waves on a SIMD no wave of the kernels beside the grid fits, so a "
                         "lighter grid lets them co-run.  Measured at 200 steps: 3 -> 2,614-2,642, "
                         "2.5 -> 2,676, 2 -> 2,669-2,688 Mvec/s; --sort --lanes 3: 1,969 -> 2,043")
    ap.add_argument("--hist-tune", default="4x256",
                    help="SPLITxTHREADS: the context histogram's launch shape when it runs off the "
                         "assignment stream (--hist-on lanes/own): split of the previous-symbol "
                         "range (LDS per workgroup 128 KB / split) x workgroup threads, so its "
                         "workgroups fit beside the assignment grid (pqh_ctx_set_tuning)")
    ap.add_argument("--split-cus", type=int, default=0,
                    help="> 0: the code-table, encode and decode streams on this many compute "
                         "units, the assignment stream on the others (disjoint CU masks)")
    ap.add_argument("--tbufs", type=int, default=2,
                    help="code-table sets per table lane when --elanes > 0")
    ap.add_argument("--a-priority", action="store_true",
                    help="run the assignment stream at high priority")
    ap.add_argument("--extra-slots", type=int, default=3,
                    help="code/count buffers beyond one per lane")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend (nccl = RCCL; gloo only to rehearse the "
                         "multi-rank schedule with every rank on one GPU, --one-device)")
    ap.add_argument("--shard-path", choices=["library", "python"], default="library",
                    help="world > 1: the library's two-phase pqh_shard_encode (C ABI, RCCL "
                         "hooks; default) or the Python composition of the same steps")
    ap.add_argument("--dist-rehearse", action="store_true",
                    help="run the multi-rank pipeline (process group, collectives, shard "
                         "phases) even with one rank: a rehearsal of the RCCL route on a "
                         "one-GPU box (launch through torch.distributed.run)")
    ap.add_argument("--shard-groups", choices=["lanes", "one"], default="one",
                    help="world > 1, library path: a process group (RCCL communicator, its own "
                         "stream) per table lane for phase 1 and per encode stream for phase 2, "
                         "so a collective waits only for its own lane's earlier work; 'one' "
                         "(default): every collective on the default group, in issue order on "
                         "one stream, phase 2 issued 'lanes x table sets - 1' batches late "
                         "(2,563 vs 2,558 Mvec/s in the one-rank rehearsal, fewer communicators)")
    ap.add_argument("--write-on", choices=["encode", "tables"], default="encode",
                    help="world > 1, library path: phase 2 (length all-gather, offsets, write) "
                         "on the encode stream, or on the batch's table lane right after its "
                         "tables, the encode stream then only decoding (needs --shard-groups "
                         "lanes; measured 2,452 vs 2,558 Mvec/s in the one-rank rehearsal)")
    ap.add_argument("--a-queue", choices=["auto", "pool", "own"], default="auto",
                    help="stream A on torch's default stream (from HIP's pool of hardware "
                         "queues, which more than 4 streams share) or on an all-CU CU-masked "
                         "stream with a hardware queue of its own (auto = own: one rank "
                         "2,873-2,905 vs 2,859-2,880 Mvec/s at 20 steps; with world > 1 RCCL's "
                         "stream is a fifth, and a lane sharing A's queue stalled it)")
    ap.add_argument("--nccl-priority", choices=["normal", "high"], default="normal",
                    help="--shard-groups lanes over RCCL: the groups' internal streams at "
                         "normal or high priority")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank uses GPU 0 (schedule rehearsal on a one-GPU box)")
    ap.add_argument("--lut-on", choices=["lanes", "assign"], default="lanes",
                    help="where a batch's decode tables are built: on its table lane after the "
                         "trees, or on the assignment stream --lut-lag batches later")
    ap.add_argument("--lut-lag", type=int, default=2)
    ap.add_argument("--pair-tables", action="store_true",
                    help="a table lane builds two consecutive batches' code tables in one "
                         "tree launch (pqh_tables_build_pair)")
    ap.add_argument("--fuse-tables", action="store_true",
                    help="each batch's Huffman trees and decode tables in one launch "
                         "(pqh_tables_build; context tables), except the run's last batch, "
                         "whose encode may start after its trees: 2,887-2,929 against "
                         "2,902-2,977 Mvec/s at 20 steps, 3,113-3,140 against 3,088-3,136 at 100")
    ap.add_argument("--timeline", action="store_true",
                    help="(diagnostic) print every timed stage's start/end in ms from the first")
    ap.add_argument("--dump", default="",
                    help="write the last batch's stitched stream and all ranks' codes to this "
                         ".npz on rank 0 (parity tests)")
    ap.add_argument("--diag-skip", default="",
                    help="(diagnostic, never a result: the JSON line is marked) comma list of "
                         "stages -- trees, luts, hist, encode, decode -- issued only for the first "
                         "batches, so a run shows what each stage costs the schedule (every batch "
                         "holds the same data, so later batches reuse valid tables / streams)")
    ap.add_argument("--table-cus", type=int, default=0,
                    help="limit each lane stream to this many CUs (0: no CU mask)")
    return ap.parse_args(argv)


GEN_CHUNK = 4_000_000   # rows generated at a time (a 125M-row shard is 64 GB)


def make_data(torch, n, d, seed, rank, device):
    """SIFT-like synthetic shard generated on the device: integer-valued floats in [0,255]
    from a Gaussian mixture with Zipf(1.1) weights.  Mixture centres
    come from `seed` (shared by all ranks), rows from (seed, rank) in chunks of GEN_CHUNK
    rows (chunk c > 0 reseeded with c), so a shard of any size is generated in place."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    centers = 1024
    torch.manual_seed(seed)    # the Gamma draw uses the default CPU generator
    mu = torch.distributions.Gamma(torch.tensor(1.2), torch.tensor(1 / 30.0)).sample((centers, d))
    mu = mu.to(device)
    w = 1.0 / torch.arange(1, centers + 1, dtype=torch.float64) ** 1.1
    w = (w / w.sum()).to(device)
    x = torch.empty((n, d), dtype=torch.float32, device=device)
    for c, r0 in enumerate(range(0, n, GEN_CHUNK)):
        r1 = min(n, r0 + GEN_CHUNK)
        g.manual_seed(seed * 1000003 + rank + c * 7919 * 1000003)
        lab = torch.multinomial(w, r1 - r0, replacement=True, generator=g)
        xc = mu[lab] + 12.0 * torch.randn((r1 - r0, d), generator=g, device=device)
        x[r0:r1] = torch.clamp(torch.round(xc), 0, 255)
        del lab, xc
    return x


def make_deep(torch, n, d, seed, rank, device):
    """Deep1B-style shard: a Gaussian mixture of 1,024 centres with
    Zipf(1.1) weights, rows normalised to unit length; generated on the device in chunks."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    mu = torch.randn((1024, d), generator=g, device=device)
    w = 1.0 / torch.arange(1, 1025, dtype=torch.float64, device=device) ** 1.1
    w = w / w.sum()
    x = torch.empty((n, d), dtype=torch.float32, device=device)
    for c, r0 in enumerate(range(0, n, GEN_CHUNK)):
        r1 = min(n, r0 + GEN_CHUNK)
        g.manual_seed(seed * 1000003 + rank + c * 7919 * 1000003)
        lab = torch.multinomial(w, r1 - r0, replacement=True, generator=g)
        xc = mu[lab] + 0.35 * torch.randn((r1 - r0, d), generator=g, device=device)
        x[r0:r1] = torch.nn.functional.normalize(xc, dim=1)
        del lab, xc
    return x


def train_centroids(torch, x, m, k, iters=4, sample=50_000, seed=7):
    """Setup only (not timed): Lloyd iterations on a device sample, float64 accumulation.
    Centroid sums are taken on the host so the setup is deterministic run to run."""
    n, d = x.shape
    ds = d // m
    g = torch.Generator(device=x.device)
    g.manual_seed(seed)
    xs = x[torch.randperm(n, generator=g, device=x.device)[:sample]].double()
    out = torch.empty((m, k, ds), dtype=torch.float32)
    for j in range(m):
        sub = xs[:, j * ds:(j + 1) * ds]
        c = sub[torch.randperm(sub.shape[0], generator=g, device=x.device)[:k]].clone()
        for _ in range(iters):
            a = torch.cdist(sub, c).argmin(1).cpu()
            s = torch.zeros((k, ds), dtype=torch.float64).index_add_(0, a, sub.cpu())
            cnt = torch.bincount(a, minlength=k).double()
            nz = cnt > 0
            c = c.cpu()
            c[nz] = s[nz] / cnt[nz, None]
            c = c.to(x.device)
        out[j] = c.float().cpu()
    return out.numpy()


def cpu_leg(orc, xs, cent, ctxm, threads, sort=False):
    """One timed pass of the CPU path on xs: assign (threads) + [stable strncmp-key sort] +
    histogram + codebooks + bit-serial encode + trie decode (single thread, as the
    reference's Huffman half)."""
    t0 = time.perf_counter()
    codes, _ = orc.pq_assign(xs, cent, threads=threads)
    if sort:
        codes = orc.sort_rows(codes)
    t1 = time.perf_counter()
    cbs = orc.build_codebooks(codes, cent.shape[1], ctxm)
    stream, bits = orc.encode(codes, cbs)
    t2 = time.perf_counter()
    dec = orc.decode(stream, len(codes), codes.shape[1], cbs)
    t3 = time.perf_counter()
    assert np.array_equal(dec, codes)
    return {"value": round(len(xs) / (t3 - t0) / 1e6, 4),
            "stages_s": {"assign": round(t1 - t0, 3), "encode": round(t2 - t1, 3),
                         "decode": round(t3 - t2, 3)}}


def cpu_baseline(x_host, cent, ctxm, sample, sort=False):
    """The reference CPU path (the oracle: a byte-exact restatement of the reference) on
    bounded samples of the shard, on this host:
      1 thread -O2 (the headline `value`), all granted threads -O2 (OpenMP over rows for the
      assignment; the Huffman half stays single-threaded like the reference's), and 1 thread
      at the reference's as-shipped -O0 -g (src/Makefile:9) on a quarter of the sample."""
    from oracle import oracle_ctypes as orc
    xs = np.ascontiguousarray(x_host[:sample])
    # the host cores this process may use (the GPU box grants a share of the machine and
    # sets OMP_NUM_THREADS to it)
    threads = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    orc.use_build("O2")
    one = cpu_leg(orc, xs, cent, ctxm, 1, sort)
    allc = cpu_leg(orc, xs, cent, ctxm, threads, sort)
    q = max(1, sample // 4)
    orc.use_build("O0")
    o0 = cpu_leg(orc, np.ascontiguousarray(xs[:q]), cent, ctxm, 1, sort)
    orc.use_build("O2")
    mode = "context" if ctxm else "non-context"
    return {"value": one["value"], "unit": "Mvec/s", "cores": 1, "kind": "port",
            "sample": f"{sample} vectors of the rank-0 shard, M={cent.shape[0]} "
                      f"K={cent.shape[1]} {mode}: oracle assign "
                      + ("+ stable strncmp-key sort " if sort else "") +
                      "+ histogram + codebooks + bit-serial encode + trie decode, single "
                      "thread -O2",
            "stages_s": one["stages_s"],
            "legs": [
                dict(one, cores=1, build="-O2", sample=sample),
                dict(allc, cores=threads, build="-O2", sample=sample,
                     note="OpenMP assignment over rows; Huffman half single-threaded"),
                dict(o0, cores=1, build="-O0 -g (as shipped)", sample=q)]}


def pcie_ms(torch, x, codes, stream_bytes):
    """PCIe-inclusive costs reported beside `value` (never part of it): pinned H2D of the
    vectors, D2H of their codes and of their stream bytes, for a 1M-row
    slice of the shard (the whole SIFT1M-shaped shard)."""
    hx = torch.empty(x.shape, dtype=x.dtype, pin_memory=True)
    hc = torch.empty(codes.shape, dtype=codes.dtype, pin_memory=True)
    hs = torch.empty(int(stream_bytes), dtype=torch.uint8, pin_memory=True)
    dsb = torch.empty(int(stream_bytes), dtype=torch.uint8, device=x.device)
    out = {}
    for name, fn in (("h2d_vectors", lambda: x.copy_(hx, non_blocking=True)),
                     ("d2h_codes", lambda: hc.copy_(codes, non_blocking=True)),
                     ("d2h_stream", lambda: hs.copy_(dsb, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t0) / 3 * 1e3, 3)
    return out


def main():
    args = parse()
    if args.hist_on == "auto":
        args.hist_on = "lanes" if args.vectors < 16_000_000 else "assign"
    # (GPU_MAX_HW_QUEUES is left to the environment, HIP's default 4: the multi-rank pipeline
    # measured 1,654 Mvec/s at 8 queues against 2,534 at 4 in the one-rank RCCL rehearsal)
    import torch
    import torch.distributed as dist
    from pq_huffman_amd import codec, shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.one_device:
        local = 0
    multi = world > 1 or args.dist_rehearse   # the multi-rank pipeline (process group)
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n = args.vectors
    d, m, k = {"sift": (128, 8, 256), "deep": (96, 16, 256), "k4096": (128, 8, 4096)}[args.config]
    ctxm = args.mode == "ctx" and k == 256     # context coding needs K = 256
    gen = make_deep if args.config == "deep" else make_data
    code_t = torch.uint8 if k <= 256 else torch.int16   # (u16 codes live in int16 tensors)
    code_bytes = 1 if k <= 256 else 2

    x = gen(torch, n, d, 0x5EED, rank, dev)
    cent = train_centroids(torch, gen(torch, 200_000, d, 0x5EED, 0, dev), m, k)
    if multi:   # one quantizer for the whole job: rank 0's centroids
        ct = torch.from_numpy(cent).to(dev)
        dist.broadcast(ct, 0)
        cent = ct.cpu().numpy()
    # Streams.  A = torch's current (default) stream: assignment + histogram of every batch.
    # `lanes` library streams (non-blocking): lane i % lanes builds batch i's code tables,
    # encodes and decodes it, with its own tables and stream buffers.  So batch i's tree
    # build (latency-bound) and encode/decode run beside the assignment of the batches after
    # it, and consecutive batches' builds overlap each other.  1 + lanes = 4 streams: with 4
    # hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default) none share a queue.
    # Serial: everything on A, in order.
    serial = args.sched == "serial" or args.no_overlap
    # stream A: torch's default stream, or (--a-priority) a high-priority stream of its own
    # --split-cus N: the table / encode / decode streams on N compute units (spread over the
    # XCDs), stream A -- the persistent assignment grid and the histogram -- on all the others
    split = args.split_cus if 0 < args.split_cus < torch.cuda.get_device_properties(dev).multi_processor_count else 0
    if split:
        torch.cuda.synchronize()   # (A gets a stream of its own: the setup's work is done)
        ctx = codec.Context(local, cus=split, complement=True)
    elif args.a_queue == "own" or (args.a_queue == "auto" and not args.a_priority):
        torch.cuda.synchronize()   # (A gets a stream of its own: the setup's work is done)
        ctx = codec.Context(local, cus=-1)
    else:
        ctx = (codec.Context(local, stream=torch.cuda.Stream(device=dev, priority=-1))
               if args.a_priority else codec.Context(local))
    sA = ctx.stream
    if args.lanes is None:   # 1 + lanes + elanes <= 4 streams: one hardware queue each
        # (k4096: the tree builds are the long stage; --sort: the sort and the histogram ride
        # on the lanes -- 1,969 vs 1,877 Mvec/s)
        # (world > 1: stream A on a hardware queue of its own, the 2 lanes, the encode stream
        # and RCCL's stream on HIP's 4 pooled queues, none shared: 2,793 Mvec/s in the one-rank
        # RCCL rehearsal; 3 lanes 1,604 with A's own queue, 2,500-2,563 without)
        args.lanes = 3 if args.config == "k4096" or args.sort else 2
    if args.elanes is None:
        args.elanes = 0 if args.config == "k4096" else 1
    nl = 1 if serial else max(1, args.lanes)
    # Lane streams are the library's own (pqh_ctx_create_cu_split; cus >= the device's CU
    # count: no CU mask).  (torch.cuda.Stream lanes measured 1,107 vs 2,250 Mvec/s: torch's
    # stream pool maps them onto the hardware queues of its other streams.)  Tensors used on
    # them are released before the contexts destroy them (teardown below).
    lanes = [ctx] if serial else [codec.Context(local, cus=split or args.table_cus or 1 << 20)
                                  for _ in range(nl)]
    # encode + decode streams: the table lanes themselves, or --elanes streams of their own
    # (then batch i's tables are built on lane i % lanes while the encode/decode streams
    # work on earlier batches, and a table lane rebuilds only after the decode that read it)
    elanes = lanes if serial or args.elanes <= 0 else [codec.Context(local, cus=split or 1 << 20)
                                                       for _ in range(args.elanes)]
    ne = len(elanes)
    pq = codec.PQ(ctx, cent)
    # more assignment streams: each with its own context (histogram workspace) and PQ object
    # (the assignment's work-queue state is per object, so launches may overlap)
    na = 1 if serial or lib_shard_req(args, multi) else max(1, args.astreams)
    actx = [ctx] + [codec.Context(local, cus=1 << 20) for _ in range(na - 1)]
    # the assignment grid's workgroups per CU, on the contexts that launch it (a library
    # caller that sets nothing gets the occupancy limit; pqh_ctx_set_tuning)
    if args.assign_wgs_per_cu > 0:
        for c in actx:
            c.set_tuning(assign_wgs_per_cu=args.assign_wgs_per_cu)
    apq = [pq] + [codec.PQ(c, cent) for c in actx[1:]]
    items = k * k if ctxm else k
    # codes / counts buffers: the assignment runs up to `slots` batches ahead of the oldest
    # batch not yet encoded
    slots = nl + max(1, args.extra_slots)
    # part-major codes (--code-layout parts): codes[s] is (m, n), part i's codes in row i
    # (world > 1: through the library's part-major shard phases, the same pipeline as one rank)
    pm = args.code_layout == "parts" and not args.sort and \
        (not multi or lib_shard_req(args, multi)) and \
        code_t == torch.uint8 and m in (8, 16) and not serial
    # (part rows padded to a multiple of 128 codes: the assignment's stores are then whole
    # 128-byte lines; with ld = n = 10^6 every odd part starts mid-line and each store
    # straddles two lines -- 1.7x the code bytes in HBM writes)
    ldp = (n + 127) // 128 * 128
    codes = [torch.empty((m, ldp), dtype=code_t, device=dev)[:, :n] if pm else
             torch.empty((n, m), dtype=code_t, device=dev) for _ in range(slots)]
    counts = [torch.zeros((m, items), dtype=torch.int32, device=dev) for _ in range(slots)]
    halo = [None] * slots
    ev_hist = [torch.cuda.Event() for _ in range(slots)]
    ev_tab = [torch.cuda.Event() for _ in range(slots)]
    ev_enc = [torch.cuda.Event() for _ in range(slots)]
    ev_trees = [torch.cuda.Event() for _ in range(slots)]
    lut_a = args.lut_on == "assign" and not serial
    dl = max(1, min(args.lut_lag, nl * (1 if elanes is lanes else max(1, args.tbufs)) - 1)) \
        if lut_a else 0
    used = [False] * slots    # slot s has held a batch (its events were recorded)
    early = [False] * slots   # batch in slot s: encode may start after its trees
    chunks = (n + args.chunk - 1) // args.chunk
    # code tables: one set per lane; two per table lane when encode/decode have streams of
    # their own, so a lane builds batch i + lanes's tables while batch i's are still read
    nbuf = 1 if elanes is lanes else max(1, args.tbufs)
    pair = args.pair_tables and not serial and elanes is not lanes
    if pair:
        nbuf = 2 * max(1, args.tbufs)   # two batches per build, double-buffered
    tabs = [codec.Tables(c, m, k, ctxm) for c in lanes for _ in range(nbuf)]
    ev_dec = [torch.cuda.Event() for _ in tabs]    # last decode that read tabs[t]

    def lane_of(i):
        return (i // 2) % nl if pair else i % nl

    def tab_index(i):
        if pair:   # lane (i // 2) % nl, pair buffer (i // 2 // nl) % (nbuf / 2), member i % 2
            return lane_of(i) * nbuf + ((i // 2) // nl) % (nbuf // 2) * 2 + i % 2
        return (i % nl) * nbuf + (i // nl) % nbuf
    # world > 1 through the C ABI (pqh_shard_encode_tables on the table lane, then
    # pqh_shard_encode_write on the encode stream, or on the table lane after the tables --
    # --write-on tables): the histogram moves off the assignment stream into phase 1; each
    # in-flight batch keeps its scratch (halo row, raw-first flag)
    lib_shard = multi and args.shard_path == "library" and not serial and not args.sort
    wt = lib_shard and elanes is not lanes and args.shard_groups == "lanes" and \
        args.write_on == "tables"
    if args.write_on == "tables" and not wt:
        raise SystemExit("--write-on tables: world > 1 (or --dist-rehearse), library path, "
                         "--shard-groups lanes, encode streams of their own")
    # the streams' buffers: one per encode stream, or (wt) one per table set, guarded by
    # that set's ev_dec like the tables themselves
    nw = len(tabs) if wt else ne
    dec = [torch.empty((n, m), dtype=code_t, device=dev) for _ in elanes]
    coff = [torch.empty(chunks, dtype=torch.int64, device=dev) for _ in range(nw)]
    cprev = [torch.empty((chunks, m), dtype=torch.uint8, device=dev) if ctxm else None
             for _ in range(nw)]
    out = [torch.zeros(n * m * 56 // 8 + 64, dtype=torch.uint8, device=dev)  # worst case
           for _ in range(nw)]
    tot_dev = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(nw)]
    raw_first = shard.raw_first(rank)
    if lib_shard:
        # (--shard-groups lanes: every rank creates the groups in the same order)
        if args.shard_groups == "lanes":
            pgo = None
            if args.dist_backend == "nccl" and args.nccl_priority == "high":
                pgo = dist.ProcessGroupNCCL.Options()
                pgo.is_high_priority_stream = True

            def group():
                return dist.new_group(list(range(world)), pg_options=pgo)
            comm_t = [shard.TorchComm(world, rank, group=group()) for _ in range(nl)]
            comm_e = [shard.TorchComm(world, rank, group=group()) for _ in range(ne)]
        else:
            comm_t = [shard.TorchComm(world, rank)] * nl
            comm_e = comm_t[:1] * ne
        scratch = [shard.scratch_for(comm_t[0], m, dev) for _ in range(slots)]
        status = [0] * slots
        offs = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(nw)]
        # every batch's global length, folded by min on the writing streams: -1 (the sentinel
        # ~0) if any rank's phase 2 failed for any batch (checked after the timed region)
        shard_min = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(nw)]
    stages = ("assign", "sort", "hist", "codebook", "lut", "encode", "decode")
    if args.sort and (k > 256 or multi):
        raise SystemExit("--sort: one rank, K <= 256 (the distributed sort is shard.py's)")
    sort_tmp = torch.empty((n, m), dtype=torch.uint8, device=dev) if args.sort else None
    # sort mode: the sort of batch i runs on its table lane (after the assignment), so the
    # assignment stream carries the assignments only; the histogram follows it there
    sort_on_lane = args.sort and args.sort_on == "lanes" and not serial
    # (one rocPRIM-path scratch per lane when the lanes sort concurrently)
    sort_tmps = [torch.empty((n, m), dtype=torch.uint8, device=dev) for _ in lanes] \
        if sort_on_lane else None
    events = []          # (stage, start, end) of timed steps, read after the timed region
    acc = {s: 0.0 for s in list(stages) + ["collectives"]}
    state = {"timed": False}

    ev_pool = []         # timing events made before the timed region (not while issuing)

    def rec(name, stream):
        # the assignment's events over the timed steps (the roofline's kernel time), the other
        # stages' over the timed steps too (--stage-events timed) or the untimed ones after
        every = args.assign_event_every
        asg_ev = name == "assign" and every > 0 and state.get("step", 0) % every == 0
        timed_ev = state["timed"] and (asg_ev or (name != "assign" and args.stage_events == "timed"))
        after_ev = state.get("after") and (name != "assign" or every <= 0)
        if not (timed_ev or after_ev):
            return None
        e0, e1 = ev_pool.pop() if ev_pool else (torch.cuda.Event(enable_timing=True),
                                                torch.cuda.Event(enable_timing=True))
        e0.record(stream)
        events.append((name, e0, e1))
        return e1

    def done(e1, stream):
        if e1 is not None:
            e1.record(stream)

    hist_on_lane = (args.hist_on == "lanes" or sort_on_lane) and not serial
    # --hist-on own: the histogram of batch i on a stream of its own, after batch i's
    # assignment, so stream A carries the assignments only
    hctx = codec.Context(local, cus=1 << 20) if args.hist_on == "own" and not serial else None
    hsplit, hthreads = (int(v) for v in args.hist_tune.lower().split("x"))
    for c in ([hctx] if hctx is not None else lanes if hist_on_lane else []):
        c.set_tuning(hist_split=hsplit, hist_block=hthreads)
    ev_asg = [torch.cuda.Event() for _ in range(slots)]
    # the split histogram: partial counts per slot (the assignment stream writes slot s's while
    # a lane may still reduce another's)
    # (world > 1, library path: the partials on stream A without the halo; phase 1 reduces
    # them on the table lane and adds the shard-boundary pair -- pqh_shard_encode_tables_parts)
    hist_split = args.hist_split == "on" and ctxm and not serial and not hist_on_lane and \
        (not lib_shard or pm) and code_t == torch.uint8
    hparts = [torch.empty(codec.histogram_partial_bytes(n, m, k), dtype=torch.uint8, device=dev)
              for _ in range(slots)] if hist_split else None
    parts = torch.arange(m, device=dev)
    ones_m = torch.ones(m, dtype=torch.int32, device=dev)

    def wait(stream, ev):
        """stream waits for ev -- unless the host sees ev already complete (a slot's previous
        batch, several steps back): a cross-stream wait is a barrier packet on the waiting
        queue, ~7-15 us of stream time per wait in the profiled schedule"""
        if not ev.query():
            stream.wait_event(ev)

    def hist(s, c, st):
        """batch s's symbol histogram on stream st (context c); with hist_split only its
        partial counts (the lane reduces them, hist_reduce)"""
        if used[s]:                  # the slot's previous batch: tables built (counts free)
            wait(st, ev_tab[s])
        e = rec("hist", st)
        if hist_split and pm:
            codec.histogram_partial_parts(c, codes[s], n, k, hparts[s], prev_row=halo[s])
        elif hist_split:
            codec.histogram_partial(c, codes[s], k, hparts[s], prev_row=halo[s])
        elif pm:
            codec.histogram_parts(c, codes[s], n, k, ctxm, prev_row=halo[s], counts=counts[s],
                                  accumulate=False)
        else:
            codec.histogram(c, codes[s], k, ctxm, prev_row=halo[s], counts=counts[s],
                            accumulate=False)        # overwrites: no zeroing pass
        done(e, st)

    def hist_reduce(s, c):
        """the second half of batch s's split histogram, on the current (lane) stream"""
        if hist_split:
            codec.histogram_reduce(c, hparts[s], n, m, k, counts[s])

    def reduce(s):
        """batch s's histogram all-reduce, issued on the current stream (a table lane): RCCL
        waits for that stream and that stream for RCCL, so the assignment stream never
        waits for the all-reduce"""
        tc = time.perf_counter()
        shard.reduce_counts(counts[s], world)
        acc["collectives"] += time.perf_counter() - tc if state["timed"] else 0.0

    def front_lib(i):
        """world > 1, library path: batch i's assignment on A, then phase 1 of
        pqh_shard_encode (halo, histogram, all-reduce, code tables) on its lane"""
        s, j = i % slots, lane_of(i)
        c = lanes[j]
        sL = c.stream
        with torch.cuda.stream(sA):
            if used[s]:              # the slot's previous batch: encoded (codes[s] free)
                wait(sA, ev_enc[s])
            e = rec("assign", sA)
            if pm:
                pq.assign_parts(x, codes[s], ctx=ctx)
            else:
                pq.assign(x, codes[s], ctx=ctx)
            done(e, sA)
            if hist_split:           # the partial pair counts, as at one rank (no halo yet)
                hist(s, ctx, sA)
            ev_hist[s].record(sA)
        with torch.cuda.stream(sL):
            sL.wait_event(ev_hist[s])
            ti = tab_index(i)
            if elanes is not lanes:              # tabs[ti] free: its last decode is done
                wait(sL, ev_dec[ti])
            e = rec("codebook", sL)
            tc = time.perf_counter()
            status[s] = shard.shard_encode_tables(c, comm_t[j], codes[s], tabs[ti], counts[s],
                                                  scratch[s], first_row=rank * n,
                                                  parts_n=n if pm else None,
                                                  partials=hparts[s] if hist_split else None)
            acc["collectives"] += time.perf_counter() - tc if state["timed"] else 0.0
            done(e, sL)
            if wt:   # phase 2 here, after the tables, on the lane's own process group
                e = rec("encode", sL)
                tc = time.perf_counter()
                write_lib(i, c, comm_t[j], ti)
                acc["collectives"] += time.perf_counter() - tc if state["timed"] else 0.0
                done(e, sL)
                ev_enc[s].record(sL)
            ev_tab[s].record(sL)
        used[s] = True

    def write_lib(i, c, comm, w):
        """phase 2 of pqh_shard_encode for batch i on c's stream, into write buffer w"""
        s = i % slots
        shard.shard_encode_write(c, comm, codes[s], tabs[tab_index(i)], out[w], args.chunk,
                                 coff[w], cprev[w], offs[w], scratch[s], status[s],
                                 first_row=rank * n, parts_n=n if pm else None)
        tot_dev[w].copy_(shard.scratch_shard_bits(scratch[s], world, m))
        torch.minimum(shard_min[w], offs[w][1:], out=shard_min[w])
        state["goff"] = offs[w][:1]

    diag = set(x for x in args.diag_skip.replace("+", ",").split(",") if x)

    def skip(stage):   # (--diag-skip: the stage after the first batches)
        return stage in diag and state.get("issued", 0) > 2 * slots

    def front(i):
        """batch i: assignment + histogram on A, then its code tables on its lane"""
        state["issued"] = state.get("issued", 0) + 1
        if lib_shard:
            return front_lib(i)
        s, j = i % slots, lane_of(i)
        c = lanes[j]
        sL = c.stream
        cF = actx[i % na]            # the stream of assignment + histogram
        sF = cF.stream
        with torch.cuda.stream(sF):
            if used[s]:              # the slot's previous batch: encoded (codes[s] free) ...
                wait(sF, ev_enc[s])
            e = rec("assign", sF)
            if pm:
                apq[i % na].assign_parts(x, codes[s], ctx=cF)
            else:
                apq[i % na].assign(x, codes[s], ctx=cF)
            done(e, sF)
            if args.sort and not sort_on_lane:   # stable strncmp-key sort (in place)
                e = rec("sort", sF)
                codec.sort_rows(cF, codes[s], sort_tmp)
                done(e, sF)
            halo[s] = None
            # (the run's last batch: its histogram on this stream, which the drain leaves
            # idle, instead of on the lane in front of its tables)
            lane_hist = hist_on_lane and (sort_on_lane or i != state["nsteps"] - 1)
            if hctx is not None:
                ev_asg[s].record(sF)
            elif skip("hist"):
                ev_hist[s].record(sF)
            elif not lane_hist:   # (the shard-boundary pair is added on the lane)
                hist(s, cF, sF)
                ev_hist[s].record(sF)
            else:
                ev_hist[s].record(sF)
        if hctx is not None:
            sH = hctx.stream
            with torch.cuda.stream(sH):
                sH.wait_event(ev_asg[s])
                hist(s, hctx, sH)
                ev_hist[s].record(sH)
        with torch.cuda.stream(sL):
            sL.wait_event(ev_hist[s])
            if not skip("hist"):
                hist_reduce(s, c)
            # the one-row halo all-gather on the lane too, so the assignment stream never
            # waits for RCCL; the pair (previous shard's last row, first row) is one more
            # count per part, exactly what pqh_histogram's prev_row adds
            tc = time.perf_counter()
            halo[s] = shard.exchange_halo(codes[s][-1], world, rank) if ctxm and not pm else None
            acc["collectives"] += time.perf_counter() - tc if state["timed"] else 0.0
            if sort_on_lane:         # the batch's sort, on its lane, before its histogram
                e = rec("sort", sL)
                codec.sort_rows(c, codes[s], sort_tmps[j])
                done(e, sL)
            if lane_hist and not skip("hist"):
                hist(s, c, sL)
            elif halo[s] is not None:
                cs = counts[s]
                cs.index_put_((parts, halo[s].long() * k + codes[s][0].long()), ones_m,
                              accumulate=True)
            reduce(s)
        used[s] = True
        if pair and i % 2 == 0 and i != state["nsteps"] - 1:
            return                   # built with batch i + 1 (its partner)
        if pair and i % 2 == 1:
            with torch.cuda.stream(sL):
                s0, t0i, ti = (i - 1) % slots, tab_index(i - 1), tab_index(i)
                wait(sL, ev_dec[t0i])
                wait(sL, ev_dec[ti])
                e = rec("codebook", sL)
                if i == state["nsteps"] - 1 and args.drain_trees != "default":
                    tabs[t0i].build(counts[s0], c, trees=args.drain_trees)   # the drain
                    tabs[ti].build(counts[s], c, trees=args.drain_trees)
                else:
                    tabs[t0i].build_pair(counts[s0], tabs[ti], counts[s], c)
                done(e, sL)
                ev_tab[s0].record(sL)
                ev_tab[s].record(sL)
            return
        with torch.cuda.stream(sL):
            ti = tab_index(i)
            if elanes is not lanes:              # tabs[ti] free: its last decode is done
                wait(sL, ev_dec[ti])
            e = rec("codebook", sL)
            # GPU trees + lookup tables, no host trip.  --drain-trees / --fill-trees pick
            # another builder for the run's last batch (built after the assignment stream is
            # done) and the lanes' first batches.
            tr = None
            if i == state["nsteps"] - 1 and args.drain_trees != "default":
                tr = args.drain_trees
            elif i < nl and args.fill_trees != "default":
                tr = args.fill_trees
            if lut_a:   # trees here, the decode tables on A dl batches later (lut())
                tabs[ti].build_trees(counts[s], c, trees=tr)
                done(e, sL)
                ev_trees[s].record(sL)
            else:
                # trees, then the decode tables: with the group builder the encode tables
                # are complete after the trees (encode_ready), so the encode stream waits
                # for ev_trees only and runs beside the decode-table build
                # (the run's last batch always: its encode is on the drain's critical path)
                split = not args.fuse_tables or args.encode_after == "trees" or \
                    i == state["nsteps"] - 1 or skip("trees") or skip("luts")
                if not split:   # one launch: each tree group builds its decode tables too
                    tabs[ti].build(counts[s], c, trees=tr)
                    early[s] = False
                    ev_trees[s].record(sL)
                else:
                    if not skip("trees"):
                        tabs[ti].build_trees(counts[s], c, trees=tr)
                    early[s] = tabs[ti].encode_ready()
                    ev_trees[s].record(sL)
                    if not skip("luts"):
                        tabs[ti].build_luts(c)
                done(e, sL)
                ev_tab[s].record(sL)
        if lut_a and i >= dl:
            lut(i - dl)

    def lut(i):
        """batch i's decode tables on the assignment stream (which has slack: it waits for
        free code buffers), after its trees on the lane"""
        s = i % slots
        with torch.cuda.stream(sA):
            sA.wait_event(ev_trees[s])
            e = rec("lut", sA)
            tabs[tab_index(i)].build_luts(ctx)
            done(e, sA)
            ev_tab[s].record(sA)

    def back(i):
        """batch i: encode + decode on its lane (queued behind its tables) or on its
        encode/decode stream (after an event wait for its tables)"""
        s, jt = i % slots, tab_index(i)
        j = i % ne
        w = jt if wt else j   # the stream's write buffer
        c = elanes[j]
        sL = c.stream
        tj = tabs[jt]
        with torch.cuda.stream(sL):
            if elanes is not lanes:
                sL.wait_event(ev_trees[s] if early[s] and not lib_shard else ev_tab[s])
            if halo[s] is not None:   # made on the table lane: keep it until this stream's use
                halo[s].record_stream(sL)
            e = rec("encode", sL) if not wt else None
            tc = time.perf_counter()
            if wt:   # (written on the table lane after the tables)
                pass
            elif lib_shard:   # phase 2 of pqh_shard_encode: length, all-gather, offsets, write
                write_lib(i, c, comm_e[j], w)
                acc["collectives"] += time.perf_counter() - tc if state["timed"] else 0.0
            elif multi:   # place the shard in the global stream before writing it: sizes,
                # all-gather + prefix sum on the device, offset read by the kernel (no host sync)
                total = codec.encode_size(c, tj, codes[s], raw_first, halo[s])
                goff, _ = shard.bit_offsets_device(total, world, rank)
                state["goff"] = goff
                out[j][:4].zero_()   # bits before the offset belong to the previous shard
                acc["collectives"] += time.perf_counter() - tc if state["timed"] else 0.0
                codec.encode_write_at(c, tj, codes[s], out[j], goff, raw_first, halo[s],
                                      args.chunk, coff[j], cprev[j], total=tot_dev[j])
            elif skip("encode"):
                pass
            elif pm:   # the row encoder gathering each row from the part runs
                codec.encode_write_parts(c, tj, codes[s], n, out[j], 0, raw_first, halo[s],
                                         args.chunk, coff[j], cprev[j], total=tot_dev[j])
            else:
                # one pass: look-back offsets, every word stored once (no zeroing of `out`)
                codec.encode_write(c, tj, codes[s], out[j], 0, raw_first, halo[s],
                                   args.chunk, coff[j], cprev[j], total=tot_dev[j])
            done(e, sL)
            if not wt:
                ev_enc[s].record(sL)
            enc = codec.Encoded(out[w], -1, args.chunk, coff[w], cprev[w], n, raw_first)
            if elanes is not lanes and early[s] and not lib_shard:
                sL.wait_event(ev_tab[s])   # the decode tables
            e = rec("decode", sL)
            if not skip("decode"):
                codec.decode(c, tj, enc, out=dec[j])
            done(e, sL)
            ev_dec[jt].record(sL)
        state["last"] = (s, j)
        state["last_w"] = w
        state["last_tab"] = jt

    # Every dependency is an event, so batches are issued in order.  With world > 1 the
    # collectives of all streams run in issue order on the process group's one stream: batch
    # i's bit-offset all-gather (which waits for its tables) is issued after the halo and
    # histogram collectives of batch i + lag, so those never queue behind a table build.
    # (back(i) must be issued before front(i + lanes * nbuf) waits for its decode)
    lag = 0 if not multi or serial or (lib_shard and args.shard_groups == "lanes") \
        else nl * nbuf - 1
    lag = max(lag, dl)   # (back(i) is issued after lut(i))
    if pair:
        lag = max(lag, 1)    # (back(i) is issued after its pair's build)

    def run(steps):
        state["nsteps"] = steps
        state["issue_t"] = []
        for i in range(steps):
            state["issue_t"].append(time.perf_counter())
            state["step"] = i
            front(i)
            if i >= lag:
                back(i - lag)
        for i in range(max(0, steps - dl), steps) if lut_a else ():
            lut(i)
        for i in range(max(0, steps - lag), steps):
            back(i)

    def barrier():
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
            torch.cuda.synchronize()

    # Device warm-up (setup, untimed, before the warmup steps): the GPU reaches its sustained
    # clocks only after tens of milliseconds of load -- measured, 20 timed steps after 5
    # warmup steps ran at 2,430 Mvec/s and after 60 at 2,630 (the assignment 0.32 vs 0.29 ms);
    # with 40 / 100 / 200 ms of this warm-up before 5 warmup steps: 2,470-2,550 / 2,590-2,600
    # / 2,560-2,640.  The assignment kernel alone runs on the batch for --device-warmup-ms;
    # its codes are recomputed by every timed step, nothing carries over.
    dw_ms = 0.0
    alone = []   # HIP-event times of the warm-up's assignment launches (the kernel alone)
    if args.device_warmup_ms > 0:
        barrier()
        tw = time.perf_counter()
        while (time.perf_counter() - tw) * 1e3 < args.device_warmup_ms:
            evs = []
            for u in range(8):
                if u >= 4:   # (the back half of each burst: the clocks have ramped)
                    evs.append((torch.cuda.Event(enable_timing=True),
                                torch.cuda.Event(enable_timing=True)))
                    evs[-1][0].record(sA)
                if pm:
                    pq.assign_parts(x, codes[0], ctx=ctx)
                else:
                    pq.assign(x, codes[0], ctx=ctx)
                if u >= 4:
                    evs[-1][1].record(sA)
            torch.cuda.synchronize()
            alone = [a.elapsed_time(b) for a, b in evs]   # (the last burst's)
        dw_ms = (time.perf_counter() - tw) * 1e3
    run(args.warmup)
    ev_pool.extend((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.steps * len(stages)))
    barrier()
    state["timed"] = True
    t0 = time.perf_counter()
    run(args.steps)
    t_issue = time.perf_counter() - t0          # host time to issue the K steps
    barrier()
    elapsed = time.perf_counter() - t0
    state["timed"] = False
    if args.stage_events == "after":
        # the other stages' events, in untimed steps of the same schedule (an event record is
        # a packet on its stream: inside the timed steps they would cost stream time)
        ev_pool.extend((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(max(args.steps, 20) * len(stages)))
        state["after"] = True
        run(max(args.steps, 20))
        barrier()
        state["after"] = False   # (the checks below use the last batch of these steps)
    nev = {s: 0 for s in acc}
    for name, e0, e1 in events:
        acc[name] += e0.elapsed_time(e1) / 1e3
        nev[name] += 1
    for name in acc:   # per-batch averages over the recorded launches
        if name != "collectives" and nev[name]:
            acc[name] *= args.steps / nev[name]
    if args.timeline and rank == 0 and events:
        f0 = events[0][1]
        for i, (name, e0, e1) in enumerate(events):
            print(f"TL {i:3d} {name:9s} {f0.elapsed_time(e0):8.3f} {f0.elapsed_time(e1):8.3f}",
                  file=sys.stderr)
    if multi:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    s_last, j_last = state["last"]
    w_last = state["last_w"]

    # correctness after timing (not timed): exact round trip of the last batch, status words
    for t in tabs:
        t.status()
    for c in elanes:
        codec.decode_status(c)
        codec.encode_status(c)
    rows_last = codec.transpose_codes(ctx, codes[s_last], n) if pm else codes[s_last]
    assert torch.equal(dec[j_last], rows_last), "round trip mismatch"
    if world == 1 and not serial:
        # the last batch's stream, re-encoded from its rows by the row-major encoder
        # (pqh_encode_write, the path tests/test_gpu_fullsize.py pins to the oracle on all 1M
        # rows) with the same tables: every stream byte, the bit count and the chunk index
        # must agree, so a wrong but self-consistent timed stream cannot pass
        tl = tabs[state["last_tab"]]
        ref_out = torch.empty_like(out[w_last])
        ref_coff = torch.empty_like(coff[w_last])
        ref_prev = torch.empty_like(cprev[w_last]) if ctxm else None
        ref_tot = torch.zeros(1, dtype=torch.int64, device=dev)
        codec.encode_write(ctx, tl, rows_last, ref_out, 0, raw_first, None, args.chunk, ref_coff,
                           ref_prev, total=ref_tot)
        codec.encode_status(ctx)
        nbits = int(ref_tot.item())
        assert int(tot_dev[w_last].item()) == nbits, "stream length != row-path re-encode"
        assert torch.equal(out[w_last][:(nbits + 7) // 8], ref_out[:(nbits + 7) // 8]), \
            "stream bytes != row-path re-encode"
        assert torch.equal(coff[w_last], ref_coff), "chunk index != row-path re-encode"
        if ctxm:
            assert torch.equal(cprev[w_last], ref_prev), "chunk context rows != row-path re-encode"
        del ref_out, ref_coff, ref_prev, ref_tot
    if lib_shard:   # every rank's pqh_shard_encode_write succeeded (no sentinel length)
        shard.status(elanes[j_last], offs[w_last])
        for j, sm in enumerate(shard_min):   # ... for every batch, not only the last
            assert int(sm.item()) >= 0, f"a rank's shard encode failed (encode stream {j})"
    rerank = pq.rerank_count(ctx)
    bits_per_vec = int(tot_dev[w_last].item()) / n

    if args.dump:   # the last batch's shard stream + codes, gathered to rank 0 (tests)
        nb = (int(tot_dev[w_last].item()) + 7) // 8 + 8
        goff = int(state["goff"].item()) if multi else 0
        mine = {"codes": rows_last.cpu().numpy(), "bits": int(tot_dev[w_last].item()),
                "goff": goff, "buf": out[w_last][:nb].cpu().numpy(), "x": x.cpu().numpy()}
        allp = [None] * world
        if world > 1:
            dist.all_gather_object(allp, mine)
        else:
            allp = [mine]
        if rank == 0:
            total = sum(p["bits"] for p in allp)
            stitched = shard.stitch_np([(p["buf"], p["goff"], p["bits"]) for p in allp], total)
            # (+ every rank's input rows and the job's centroids: the tests check the codes
            # against the oracle's assignment too, not only the stream of these codes)
            np.savez(args.dump, stream=stitched, bits=np.int64(total),
                     codes=np.concatenate([p["codes"] for p in allp]),
                     x=np.concatenate([p["x"] for p in allp]), cent=cent)

    if rank == 0:
        t_assign = acc["assign"] / args.steps
        vec_read, vec_write = 4 * d, m * code_bytes
        achieved = (vec_read + vec_write) * n / t_assign / 1e9
        akern = ASSIGN_KERNEL[args.config]
        traffic, traffic_src, prof_avg_us = pmc_traffic(akern, profile_tag(args.config, args.sort, args.vectors))
        t_enc = (acc["assign"] + acc["hist"] + acc["codebook"] + acc["lut"] + acc["encode"]) / args.steps
        tf = 2.0 * k * d * n / t_assign / 1e12   # algorithmic: 2 K D flop per vector
        workload = {
            "sift": f"SIFT1M-shaped: {n:,} x 128-d fp32 per GPU, M=8, K=256, ",
            "deep": f"Deep1B-style (BASELINE configs[3]): {n:,} x 96-d unit-norm fp32 per GPU, "
                    "M=16, K=256 (dsub 6), ",
            "k4096": f"large codebook (BASELINE configs[4]): {n:,} x 128-d fp32 per GPU, M=8, "
                     "K=4096 (12-bit codes stored u16), "}[args.config]
        data = {
            "sift": "synthetic SIFT-like (integer-valued fp32 in [0,255], Gaussian mixture, "
                    "Zipf(1.1) weights), generated on device",
            "deep": "synthetic Deep-like (Gaussian mixture of 1,024 centres, Zipf(1.1) weights, "
                    "rows normalised to unit length), generated on device",
            "k4096": "synthetic SIFT-like (integer-valued fp32 in [0,255], Gaussian mixture, "
                     "Zipf(1.1) weights), generated on device"}[args.config]
        res = {
            "metric": (f"DIAGNOSTIC (stages skipped: {args.diag_skip}; not a result) "
                       if args.diag_skip else "") +
            (METRIC if args.config == "sift" else
             f"Mvec/s encode+decode round-trip, {d}-d fp32 M={m} K={k}; % HBM-read roofline"),
            "value": round(world * n * args.steps / elapsed / 1e6, 2),
            "unit": "Mvec/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "device_warmup_ms": round(dw_ms, 1),
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data + "; centroids from 4 Lloyd iterations on a 50k sample (setup, untimed)",
            "config": {"workload": workload
                                   + ("order-1 context Huffman (reference default coding), "
                                      if ctxm else "non-context Huffman, ")
                                   + ("rows sorted by the strncmp key (the reference's default "
                                      "mode)" if args.sort else "no sort"),
                       "sort": bool(args.sort),
                       "code_layout": "parts" if pm else "rows",
                       # the K = 256 assignment grid's workgroups per CU set on the assignment
                       # contexts (pqh_ctx_set_tuning; a library caller that sets nothing gets
                       # the occupancy limit, 3)
                       "assign_wgs_per_cu": (args.assign_wgs_per_cu if args.assign_wgs_per_cu > 0
                                             else "library default"),
                       "histogram_stream": "assignment" if not (hist_on_lane or hctx) else
                                           ("table lanes" if hist_on_lane else "own"),
                       "histogram_launch": (args.hist_tune if (hist_on_lane or hctx) else
                                            "library default"),
                       "vectors_per_gpu": n, "job_vectors_per_step": world * n,
                       # which BASELINE.json configuration this line measures (weak scaling:
                       # every rank encodes its own shard of vectors_per_gpu rows per step)
                       "baseline_config": baseline_config(args.config, n, world,
                                                          args.dist_rehearse),
                       "d": d, "m": m, "k": k,
                       "mode": "ctx" if ctxm else "noctx",
                       "chunk_vectors": args.chunk, "parallelism": f"dp{world} row shards"
                       + (" (--dist-rehearse: the multi-rank pipeline and its collectives at "
                          "one rank)" if args.dist_rehearse else ""),
                       "schedule": ("serial" if serial else
                                    "lanes: assignment + histogram " +
                                    ("partial counts " if hist_split else "") +
                                    "of every batch on one stream; batch i's " +
                                    ("histogram reduce and " if hist_split else "") +
                                    f"code tables on table lane i % {nl}" +
                                    ("" if elanes is lanes else
                                     f", its encode and decode on {ne} stream(s) of their own") +
                                    ", beside the assignment of the next batches; every timed "
                                    "step runs all five stages and the pipeline fills and "
                                    "drains inside the timed region")},
            "roofline": {"kernel": akern,
                         # `bound`: the roofline the fraction is taken against (the contract's
                         # HBM read roofline); `measured_limiter`: what the PMC counters show
                         # limits the kernel
                         "bound": "hbm",
                         "measured_limiter": "VALU issue: the exact top-2 reduction costs "
                                             "~1 VALU per score (270 VALU per 32-vector block, "
                                             "profiles/r6_assign_sq.txt); alone the kernel runs "
                                             "at ~74 % of its VALU-issue bound, and in the "
                                             "schedule it shares the SIMDs with the side "
                                             "kernels -- not HBM (traffic 1.05x the "
                                             "algorithmic bytes)",
                         "mfma_tflops_algorithmic": round(tf, 1),
                         # of the dense bf16 peak (~2.5 PF/s); each fp32 product costs two or
                         # three bf16 MFMA passes (the hi/lo split), so issued MFMA work is 2-3x
                         "mfma_frac_bf16_dense": round(tf / 2500.0, 4),
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "bytes_per_vector": vec_read + vec_write,
                         "avg_ms": round(t_assign * 1e3, 4),
                         # rocprofv3 kernel-trace average of this bench command (dispatch
                         # begin -> end); avg_ms above is HIP events around the launch on its
                         # stream, which also count the wait for CUs held by the lanes
                         "profile_avg_ms": (round(prof_avg_us / 1e3, 4)
                                            if prof_avg_us is not None else None),
                         # the same kernel alone (the device warm-up's last launches, HIP
                         # events): frac is the in-schedule figure, where it shares the GPU
                         # with the lanes' kernels by design
                         "alone_avg_ms": (round(sum(alone) / len(alone), 4) if alone else None),
                         "alone_frac": (round((vec_read + vec_write) * n / (sum(alone) / len(alone) * 1e-3)
                                              / 1e9 / HBM_PEAK_GBS, 4) if alone else None)},
            "stages_ms": {s: round(v / args.steps * 1e3, 4) for s, v in acc.items()
                          if (s != "sort" or args.sort) and (s != "lut" or lut_a)},
            "stages_note": ("per-stage HIP-event times on their own streams (the assignment's "
                            "over the timed steps, the others over untimed steps of the same "
                            "schedule after them, --stage-events)" +
                            ("" if serial else "; the stages of consecutive batches run "
                             "concurrently, so they sum to more than ms_per_step")),
            # encode-side HBM-read roofline = 512 B/vec x N / t_encode / 8 TB/s, with
            # t_encode = the summed encode-side stage times of one batch (latency view) and,
            # for the throughput view, the whole round-trip step time
            "encode_read_roofline_frac": round(vec_read * n / t_enc / 1e9 / HBM_PEAK_GBS, 4),
            "roundtrip_read_roofline_frac": round(
                vec_read * n * world * args.steps / elapsed / 1e9 / HBM_PEAK_GBS / world, 4),
            "host_issue_ms_per_step": round(t_issue / args.steps * 1e3, 3),
            # the longest pause between two steps' issue (a host stall starves the GPU)
            "host_issue_max_gap_ms": round(max((b - a for a, b in zip(state["issue_t"],
                                                                      state["issue_t"][1:])),
                                               default=0.0) * 1e3, 3),
            "bits_per_vector": round(bits_per_vec, 3),
            # the decode's chunk index, written by the encoder beside the stream (HBM-resident
            # here; huffman_indices.bin itself is unchanged): offset + context row per chunk
            "chunk_index_bytes_per_vector": round((8 + (m * code_bytes if ctxm else 0))
                                                  / args.chunk, 3),
            # what a stored batch occupies with its decode index: the stream plus the chunk
            # index (the index is the price of the short decode chains that --chunk buys)
            "stream_plus_index_bytes_per_vector": round(
                bits_per_vec / 8 + (8 + (m * code_bytes if ctxm else 0)) / args.chunk, 3),
            "rerank_fraction": round(rerank / (n * m), 6),
        }
        if world == 1:
            # (after the timed region, on a scratch copy of a 1M-row slice)
            r1 = min(n, 1_000_000)
            res["pcie_ms"] = pcie_ms(torch, x[:r1].clone(), rows_last[:r1],
                                     (bits_per_vec * r1 + 7) // 8)
            res["pcie_ms"]["rows"] = r1
        if not args.no_cpu_baseline and world == 1:
            sample = max(1000, args.cpu_sample * 256 // k)   # ~the same CPU time at any K
            xh = x[:sample].cpu().numpy()
            res["cpu_baseline"] = cpu_baseline(xh, cent, ctxm, sample, args.sort)
            res["cpu_baseline"]["host_cpu"] = _cpu_name()
            res["cpu_baseline"]["nproc"] = os.cpu_count()
        print(json.dumps(res), flush=True)
    # Teardown in a fixed order while HIP is alive.  The halo rows were used on the lane
    # streams (record_stream): torch's allocator records an event on those streams when such
    # a tensor is freed, so they are freed -- and the allocator's events drained -- while the
    # streams exist; then tables, codebook and contexts (which destroy the lane streams).
    halo[:] = [None] * slots
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    for t in tabs:
        t.close()
    for q in apq:
        q.close()
    for c in {id(c): c for c in list(lanes) + list(elanes) + list(actx) +
              ([hctx] if hctx is not None else [])}.values():
        c.close()
    if multi:
        dist.barrier()
        dist.destroy_process_group()


def baseline_config(config, n, world, rehearse=False):
    """the BASELINE.json configuration a bench line measures"""
    if rehearse and world == 1:
        return ("the multi-rank pipeline rehearsed with one rank (--dist-rehearse) on "
                + baseline_config(config, n, 8 if n < 125_000_000 else 1))
    if config == "deep":
        return "configs[3] (Deep-style 96-d, M=16)" + (f", {world} ranks" if world > 1 else "")
    if config == "k4096":
        return "configs[4] (K=4096)" + (f", {world} ranks" if world > 1 else "")
    if n >= 125_000_000:
        return (f"configs[2] per-rank shard (1B rows / 8 GPUs = 125M per rank); {world} rank(s) "
                f"x {n:,} rows = {world * n:,} rows per step")
    if world == 1:
        return "configs[1] (SIFT1M: 1M x 128-d, M=8, K=256) -- the headline"
    return (f"configs[1] weak-scaled: {world} ranks x {n:,} rows per step; configs[2]'s "
            "1B-row job is this path at --vectors 125000000 per rank")


def _cpu_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
