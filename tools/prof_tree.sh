#!/bin/bash
# Tree-mode evidence (GPU box): kernel trace + stats of tools/tree_bench.py at 1M rows
# (device tree order, encode, decode) -> gpurun_out/prof_tree/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/prof_tree; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 "$R/tools/tree_bench.py" > "$OUT/kt.log" 2>&1
