#!/bin/bash
# Collect one configuration's evidence for profiles/ (run on the GPU box from the repo root):
#   1. the bench line itself (no profiler attached)        -> $OUT/bench.log
#   2. kernel trace + per-kernel stats of the same command -> $OUT/kt/
#   3. the HBM byte counters, each in a pass of its own (FETCH_SIZE and WRITE_SIZE do not fit
#      one TCC pass; MI355X_MICROARCH.md "HBM")           -> $OUT/fetch/, $OUT/write/
# then `python profiles/summarize.py <tag>` writes profiles/<tag>_{bench.json,kernel_stats.csv,
# pmc_summary.json}.
# usage: bash profiles/collect.sh <tag, e.g. r3_sift> [bench args...]
set -euo pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/write.log" 2>&1
echo "profiles collected under $OUT"
