"""Summarise one configuration's collection (gpurun_out/prof_<tag>, profiles/collect.sh) into
profiles/:
  <tag>_bench.json         the unprofiled bench JSON line
  <tag>_kernel_stats.csv   the --kernel-trace --stats summary (copied)
  <tag>_pmc_summary.json   per-kernel average duration and HBM bytes per launch:
                           FETCH_SIZE x 2 (gfx950 reports half of wide streaming reads,
                           MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both KB -> bytes
usage: python profiles/summarize.py <tag>"""
import collections
import csv
import json
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def short(name):
    m = re.search(r"namespace\)::(\w+)", name)
    if m:
        t = re.search(r"::\w+<([^>]*)>", name)
        return m.group(1) + (f"<{t.group(1)}>" if t else "")
    return name.split("(")[0][:80]


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def bench_line(src, tag):
    """the unprofiled bench JSON line of the collection -> profiles/<tag>_bench.json"""
    path = os.path.join(src, "bench.log")
    if not os.path.exists(path):
        return
    lines = [x for x in open(path) if x.startswith("{")]
    if lines:
        with open(os.path.join(HERE, f"{tag}_bench.json"), "w") as f:
            json.dump(json.loads(lines[-1]), f, indent=1)


def fill_traffic(tag, summary):
    """the bench line was taken before its own PMC passes existed: give its roofline the
    traffic and kernel-trace average of exactly its kernel from this collection"""
    path = os.path.join(HERE, f"{tag}_bench.json")
    if not os.path.exists(path):
        return
    line = json.load(open(path))
    rf = line.get("roofline") or {}
    e = summary["kernels"].get(rf.get("kernel"))
    if not e or "hbm_bytes" not in e:
        return
    rf["traffic"] = e["hbm_bytes"]
    rf["traffic_source"] = f"profiles/{tag}_pmc_summary.json"
    rf["profile_avg_ms"] = round(e["avg_us"] / 1e3, 4)
    with open(path, "w") as f:
        json.dump(line, f, indent=1)


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    bench_line(src, tag)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"),
                os.path.join(HERE, f"{tag}_kernel_stats.csv"))
    dur = {}
    for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
        dur[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                 "pct": float(r["Percentage"])}
    fetch = per_kernel(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    out = {"source": f"gpurun_out/prof_{tag} (profiles/collect.sh)",
           "correction": "read_bytes = 2 x FETCH_SIZE(KB) x 1024 (gfx950 half-count of wide "
                         "streaming reads); write_bytes = WRITE_SIZE(KB) x 1024",
           "kernels": {}}
    for k, d in sorted(dur.items(), key=lambda kv: -kv[1]["pct"]):
        e = dict(d)
        if k in fetch:
            e["read_bytes"] = round(2 * fetch[k] * 1024)
        if k in write:
            e["write_bytes"] = round(write[k] * 1024)
        if "read_bytes" in e and "write_bytes" in e:
            e["hbm_bytes"] = e["read_bytes"] + e["write_bytes"]
        out["kernels"][k] = e
    with open(os.path.join(HERE, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    fill_traffic(tag, out)
    for k, e in list(out["kernels"].items())[:12]:
        print(k, e)


if __name__ == "__main__":
    main(sys.argv[1])
