set -o pipefail
PQH_LIB=pq_huffman_amd/lib/variants/stamps/libpqh.so timeout -k 10 120 python tools/assign_stamps.py 2>&1 | grep -v amdgpu.ids
for v in 4_4_0_1 4_4_1_1 4_3_1_1 8_2_0_1 2_4_0_1 4_5_0_1; do
  echo "== $v"; PQH_LIB=pq_huffman_amd/lib/variants/$v/libpqh.so timeout -k 10 120 python tools/bench_assign.py 20 2>&1 | grep -v amdgpu.ids
done
