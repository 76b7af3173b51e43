#!/bin/bash
# Tree-build check (diagnostic): GPU tree/codebook tests, then the table-build timing for the
# LDS build (default) and the register-heap build (PQH_TREE_IMPL=wave).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/trees_${1:-x}; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_huffman.py tests/test_tree.py tests/test_gpu_configs.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 120 python tools/bench_trees.py 2>&1 | grep -v amdgpu.ids || exit 1
PQH_TREE_IMPL=wave timeout -k 10 120 python tools/bench_trees.py 2>&1 | grep -v amdgpu.ids || exit 1
