set -o pipefail
for v in $(ls pq_huffman_amd/lib/variants); do
  echo "== $v"; PQH_LIB=pq_huffman_amd/lib/variants/$v/libpqh.so timeout -k 10 120 python tools/bench_assign.py 30 2>&1 | grep -v amdgpu.ids
done
