#!/bin/bash
# Diagnostic A/B of bench.py schedule flags (20 and 100 steps, two rounds) -> gpurun_out/benchab/
#   bash tools/gpu_benchab.sh "label:flags" ...   (NAME=VALUE words in flags go to the env)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/benchab; mkdir -p "$OUT"; cd "$R"
for r in 1 2; do
  for spec in "$@"; do
    L=${spec%%:*}; F=""; E=()
    for w in ${spec#*:}; do
      if [[ $w =~ ^[A-Z_0-9]+= ]]; then E+=("$w"); else F="$F $w"; fi
    done
    for K in 20 100; do
      env "${E[@]}" timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline $F > "$OUT/$L.$K.$r.log" 2>&1 || { tail -5 "$OUT/$L.$K.$r.log"; exit 1; }
      python - "$OUT/$L.$K.$r.log" "$L" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); st = d.get("stages_ms", {})
        print(sys.argv[2], "K", d["steps"], "value", d["value"], {k: v for k, v in st.items() if v})
PY
    done
  done
done
