#!/bin/bash
# Round-2 re-entry check: full -m gpu suite, smoke, default bench, 125M-row shard bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r2c; mkdir -p "$OUT"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -60 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
grep smoke "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench.log"
timeout -k 10 600 python bench.py --vectors 125000000 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench125m.log" 2>&1 || { tail -20 "$OUT/bench125m.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench125m.log"
