#!/bin/bash
# bench only (diagnostic): 20-step and 200-step lines + stage times -> gpurun_out/bench_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-x}; OUT=$R/gpurun_out/bench_$TAG; mkdir -p "$OUT"; cd "$R"
for st in 20 200; do
timeout -k 10 400 python bench.py --steps $st --warmup 5 --no-cpu-baseline > "$OUT/bench$st.log" 2>&1 || { tail -20 "$OUT/bench$st.log"; exit 1; }
python - "$OUT/bench$st.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); print(d["steps"], d["value"], d["ms_per_step"], d["stages_ms"])
PY
done
timeout -k 10 120 python tools/bench_trees.py 2>&1 | grep -v amdgpu.ids
