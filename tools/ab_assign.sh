#!/bin/bash
# A/B timing of the assignment kernel on the GPU box (diagnostic):
#   bash tools/ab_assign.sh <variant-dir under pq_huffman_amd/lib/variants> [rounds]
# runs the GPU PQ tests against the in-tree library, then alternates tools/bench_assign.py
# between the variant library (PQH_LIB) and the in-tree one.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$1; N=${2:-2}
mkdir -p "$R/gpurun_out"
timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_pq.py" -x -q --timeout 120 \
    --timeout-method thread > "$R/gpurun_out/gpu_pq.log" 2>&1
tail -2 "$R/gpurun_out/gpu_pq.log"
for i in $(seq "$N"); do
    echo -n "variant $V: "
    PQH_LIB=$R/pq_huffman_amd/lib/variants/$V/libpqh.so timeout -k 10 100 python "$R/tools/bench_assign.py" 50
    echo -n "in-tree:     "
    timeout -k 10 100 python "$R/tools/bench_assign.py" 50
done
