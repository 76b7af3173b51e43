#!/bin/bash
# Forest-builder evidence (GPU box): kernel trace + stats of tools/bench_forest.py at 1M rows
# (run.sh geometry) -> gpurun_out/prof_forest/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/prof_forest; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 "$R/tools/bench_forest.py" --reps 1 > "$OUT/kt.log" 2>&1
