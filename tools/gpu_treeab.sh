#!/bin/bash
# Diagnostic A/B of the tree builder inside the pipelined bench (20 and 100 steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/treeab; mkdir -p "$OUT"; cd "$R"
run() {  # label env...
  local L=$1; shift
  for K in 20 100; do
    env "$@" timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline ${BARGS:-} > "$OUT/$L.$K.log" 2>&1 || { tail -5 "$OUT/$L.$K.log"; exit 1; }
    python - "$OUT/$L.$K.log" "$L" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); print(sys.argv[2], "K", d["steps"], "value", d["value"], "stages", d.get("stages_ms"))
PY
  done
}
run base PQH_X=0
run wave PQH_TREE_IMPL=wave
run tpw8 PQH_TREE_TPW=8
run tpw32 PQH_TREE_TPW=32
run base2 PQH_X=0
