#!/bin/bash
# Diagnostic: N short profiled bench runs; per run the value and which hardware queue each
# stage's kernels ran on (rocprofv3 kernel trace Queue_Id) -> gpurun_out/qmap/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/qmap; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 ${1:-6}); do
  cd /tmp
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/r$r" -o kt --output-format csv \
      -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/r$r.log" 2>&1 || exit 1
  python3 - "$OUT" "$r" <<'PY'
import csv, collections, glob, json, sys
out, r = sys.argv[1], sys.argv[2]
v = [json.loads(l) for l in open(f"{out}/r{r}.log") if l.startswith("{")][0]
f = glob.glob(f"{out}/r{r}/**/*kernel_trace.csv", recursive=True)[0]
m = collections.defaultdict(collections.Counter)
for row in csv.DictReader(open(f)):
    for key in ("pq_assign", "hist_ctx<", "huff_trees", "enc_onepass", "dec_chunks"):
        if key in row["Kernel_Name"]:
            m[key][row["Queue_Id"]] += 1
print(r, v["value"], {k: dict(c) for k, c in m.items()}, flush=True)
PY
done
