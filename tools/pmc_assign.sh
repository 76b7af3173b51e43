#!/bin/bash
# PMC passes over the assignment-only diagnostic: bash tools/pmc_assign.sh <tag> "<ctrs>" ...
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; shift
export TMPDIR=/tmp; cd /tmp
i=0
for CTR in "$@"; do
  OUT=$R/gpurun_out/pmc_assign_${TAG}_$i; mkdir -p "$OUT"
  timeout -k 10 240 rocprofv3 --pmc $CTR -d "$OUT" -o pmc --output-format csv \
      -- python3 "$R/tools/bench_assign.py" 5 > "$OUT/log" 2>&1
  i=$((i+1))
done
