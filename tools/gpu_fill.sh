#!/bin/bash
# Diagnostic: bench wall time against the step count (pipeline fill + drain), and the
# configs[2] per-rank shard (125M rows) bench line -> gpurun_out/fill_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-x}; OUT=$R/gpurun_out/fill_$TAG; mkdir -p "$OUT"; cd "$R"
for K in 5 10 20 40 100; do
  timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline > "$OUT/k$K.log" 2>&1 || { tail -20 "$OUT/k$K.log"; exit 1; }
  python - "$OUT/k$K.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); print("K", d["steps"], "ms/step", d["ms_per_step"], "total ms", round(d["ms_per_step"] * d["steps"], 3), "value", d["value"])
PY
done
timeout -k 10 600 python bench.py --vectors 125000000 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench125m.log" 2>&1 || { tail -20 "$OUT/bench125m.log"; exit 1; }
grep '^{' "$OUT/bench125m.log" | cut -c1-400
