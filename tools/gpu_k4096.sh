#!/bin/bash
# K=4096 checks (diagnostic): the K=4096 GPU tests, then the configs[4] bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/k4096_${1:-x}; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_huffman.py -k "k4096" -x -q \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 500 python bench.py --config k4096 --steps 20 --warmup 3 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT/bench.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"]
        print(d["value"], d["ms_per_step"], d["stages_ms"], "assign", r["avg_ms"], "cpu", d.get("cpu_baseline", {}).get("value"))
PY
