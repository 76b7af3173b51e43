#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r2b; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py -x -v \
   --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for st in 20 200; do
timeout -k 10 400 python bench.py --steps $st --warmup 5 --no-cpu-baseline > "$OUT/bench$st.log" 2>&1 || { tail -20 "$OUT/bench$st.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench$st.log" | cut -c1-400
done
