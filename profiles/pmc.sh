#!/bin/bash
# One PMC pass over a short bench run: bash profiles/pmc.sh <tag> "<counters>" [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pmc_$1; CTR=$2; shift 2
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc $CTR -d "$OUT" -o pmc --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 1 "$@" > "$OUT/log" 2>&1
