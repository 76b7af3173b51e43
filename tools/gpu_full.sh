#!/bin/bash
# Full GPU check (diagnostic): pytest -m gpu, smoke, default bench line -> gpurun_out/full_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-x}; OUT=$R/gpurun_out/full_$TAG; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench.log"
