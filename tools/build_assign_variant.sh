#!/bin/bash
# One diagnostic A/B build of libpqh with the assignment kernel compiled under extra flags:
#   bash tools/build_assign_variant.sh <name> "-DPQH_ASSIGN_...=..." -> pq_huffman_amd/lib/variants/<name>/libpqh.so
# (run it after the default build: the other objects come from pq_huffman_amd/lib/obj; load the
# variant with PQH_LIB=pq_huffman_amd/lib/variants/<name>/libpqh.so)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/pq_huffman_amd/csrc; O=$R/pq_huffman_amd/lib/obj
D=$R/pq_huffman_amd/lib/variants/$1; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$R/include $2 \
   -mllvm -amdgpu-atomic-optimizer-strategy=None -c $C/hip/pqh_assign.hip -o $D/pqh_assign.o
objs=$(ls $O/*.o | grep -v '/pqh_assign.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpqh.so $objs $D/pqh_assign.o -lpthread
rm $D/pqh_assign.o
