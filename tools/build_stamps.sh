#!/bin/bash
# diagnostic build: libpqh with per-wave stamps in pq_assign_mfma -> pq_huffman_amd/lib/variants/stamps
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/pq_huffman_amd/csrc; O=$R/pq_huffman_amd/lib/obj
D=$R/pq_huffman_amd/lib/variants/stamps; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$R/include \
   -DPQH_ASSIGN_STAMPS $EXTRA -mllvm -amdgpu-atomic-optimizer-strategy=None -c $C/hip/pqh_assign.hip -o $D/pqh_assign.o
objs=$(ls $O/*.o | grep -v '/pqh_assign.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpqh.so $objs $D/pqh_assign.o -lpthread
