"""Per-kernel SQ instruction mix from tools/bench_sq_mix.sh: python tools/sq_mix_report.py <tag>"""
import csv, re, sys, glob
from collections import defaultdict
tag=sys.argv[1]
agg=defaultdict(lambda: defaultdict(float)); disp=defaultdict(set)
for f in sorted(glob.glob(f"gpurun_out/sqmix_{tag}_*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n=r["Kernel_Name"]; n=n.replace("(anonymous namespace)::",""); n=re.sub(r"^void ","",n); n=re.sub(r"\(.*","",n)[:45]
        agg[n][r["Counter_Name"]]+=float(r["Counter_Value"]); disp[(n,r["Counter_Name"])].add(r["Dispatch_Id"])
cols=["SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_INSTS_LDS","SQ_INSTS_MFMA","SQ_INSTS_SMEM","SQ_INSTS_VMEM_RD","SQ_INSTS_VMEM_WR","SQ_ACTIVE_INST_VALU","SQ_ACTIVE_INST_LDS","SQ_ACTIVE_INST_ANY","SQ_WAVES","SQ_WAVE_CYCLES","SQ_BUSY_CYCLES"]
lab=["VALU","SALU","LDS","MFMA","SMEM","VMEM_RD","VMEM_WR","ACT_VALU","ACT_LDS","ACT_ANY","WAVES","WAVE_CYC","BUSY_CYC"]
print(f"{'kernel':45s} "+" ".join(f"{c:>9s}" for c in lab))
for n,d in sorted(agg.items(), key=lambda kv:-kv[1].get("SQ_ACTIVE_INST_ANY",0)):
    vals=[]
    for c in cols:
        k=len(disp[(n,c)]) or 1
        vals.append(d.get(c,0)/k)
    print(f"{n:45s} "+" ".join(f"{v/1e6:9.3f}" for v in vals))
