#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   kernel trace + per-kernel stats of the default bench command, then the HBM byte
#   counters in their own passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
# usage: bash profiles/collect.sh <round-tag> [bench args...]
set -euo pipefail
TAG=${1:?round tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/write.log" 2>&1
echo "profiles collected under $OUT"
