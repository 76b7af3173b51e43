"""Per-dispatch PMC averages of one kernel from the passes under gpurun_out/<dir>/pmc_*/,
per 32-vector block (diagnostic): python tools/pmc_blocks.py <dir> [kernel] [blocks]."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "pq_assign_mfma"
blocks = float(sys.argv[3]) if len(sys.argv) > 3 else 1e6 * 8 / 32
agg, cnt = defaultdict(float), defaultdict(int)
for f in sorted(glob.glob(f"gpurun_out/{d}/pmc_*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
for c in sorted(agg):
    v = agg[c] / cnt[c]
    print(f"{c:28s} {v:16.0f}  per-block {v / blocks:10.2f}")
