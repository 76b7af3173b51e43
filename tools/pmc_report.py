"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_assign_<tag>_<i>/) for one kernel:
per-dispatch averages, plus per-unit values when --units is given."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    tag, kern = sys.argv[1], sys.argv[2]
    units = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    agg = defaultdict(float)
    cnt = defaultdict(int)
    for f in sorted(glob.glob(f"gpurun_out/pmc_assign_{tag}_*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]] += 1
    for c in sorted(agg):
        v = agg[c] / cnt[c]
        print(f"{c:32s} {v:16.0f} per-unit {v / units:12.2f}")


if __name__ == "__main__":
    main()
