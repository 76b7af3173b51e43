set -o pipefail
PQH_LIB=pq_huffman_amd/lib/variants/stamps/libpqh.so timeout -k 10 120 python tools/assign_stamps.py 2>&1 | grep -v amdgpu.ids
