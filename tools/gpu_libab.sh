#!/bin/bash
# Diagnostic: GPU tests of the in-tree library, then the pipelined bench alternating between
# the in-tree library and a variant (PQH_LIB) at 20 and 100 steps -> gpurun_out/libab/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/libab; mkdir -p "$OUT"; cd "$R"
V=${1:-base}; TESTS=${TESTS:-tests/test_gpu_huffman.py tests/test_gpu_configs.py tests/test_tree.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for r in 1 2; do
  for L in variant intree; do
    for K in 20 100; do
      if [ $L = variant ]; then E="PQH_LIB=$R/pq_huffman_amd/lib/variants/$V/libpqh.so"; else E="PQH_X=0"; fi
      env $E timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline > "$OUT/$L.$K.$r.log" 2>&1 || { tail -5 "$OUT/$L.$K.$r.log"; exit 1; }
      python - "$OUT/$L.$K.$r.log" "$L" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); print(sys.argv[2], "K", d["steps"], "value", d["value"], "stages", d.get("stages_ms"))
PY
    done
  done
done
