#!/bin/bash
# bench lines for BASELINE configs[3] (deep) and configs[4] (k4096) -> gpurun_out/cfg_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-x}; OUT=$R/gpurun_out/cfg_$TAG; mkdir -p "$OUT"; cd "$R"
for cfg in deep k4096; do
timeout -k 10 500 python bench.py --config $cfg --steps 20 --warmup 3 > "$OUT/bench_$cfg.log" 2>&1 || { tail -20 "$OUT/bench_$cfg.log"; exit 1; }
python - "$OUT/bench_$cfg.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"]
        print(d["config"]["workload"][:40], d["value"], d["ms_per_step"], d["stages_ms"],
              "assign", r["avg_ms"], "tflops", r["mfma_tflops_algorithmic"], "frac", r["frac"],
              "cpu", d.get("cpu_baseline", {}).get("value"))
PY
done
