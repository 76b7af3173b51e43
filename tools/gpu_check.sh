#!/bin/bash
# GPU check (diagnostic): full -m gpu suite, smoke, driver-config bench (20 steps) and a
# 200-step bench -> gpurun_out/check_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-x}; OUT=$R/gpurun_out/check_$TAG; mkdir -p "$OUT"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -60 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20.log" 2>&1 || { tail -20 "$OUT/bench20.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench20.log" | cut -c1-600
timeout -k 10 400 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/bench200.log" 2>&1 || { tail -20 "$OUT/bench200.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench200.log" | cut -c1-300
python - "$OUT/bench200.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); print("stages", d.get("stages_ms"), "assign", d["roofline"]["avg_ms"])
PY
