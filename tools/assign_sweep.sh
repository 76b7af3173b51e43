#!/bin/bash
# tools/bench_assign.py over the in-tree library and every variant (diagnostic)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for i in 1 2; do
  echo -n "in-tree: "; timeout -k 10 120 python "$R/tools/bench_assign.py" 50 2>&1 | grep -v amdgpu.ids || exit 1
  for v in $(ls "$R/pq_huffman_amd/lib/variants"); do
    echo -n "$v: "; PQH_LIB=$R/pq_huffman_amd/lib/variants/$v/libpqh.so \
      timeout -k 10 120 python "$R/tools/bench_assign.py" 50 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
