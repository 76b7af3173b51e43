#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r2a; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_fullsize.py -x -v \
   --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -8 "$OUT/tests.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench.log"
timeout -k 10 600 python bench.py --vectors 125000000 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench125m.log" 2>&1 || { tail -20 "$OUT/bench125m.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench125m.log"
