#!/bin/bash
# Diagnostic A/B builds of libpqh with extra -D flags on the assignment kernel:
#   bash tools/build_defs.sh name1 "-DFOO=1 -DBAR" name2 "-DBAZ" ...
#        -> pq_huffman_amd/lib/variants/<name>/libpqh.so
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/pq_huffman_amd/csrc; O=$R/pq_huffman_amd/lib/obj
while [ $# -gt 1 ]; do
  N=$1; F=$2; shift 2
  D=$R/pq_huffman_amd/lib/variants/$N; mkdir -p $D
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$R/include \
     $F -mllvm -amdgpu-atomic-optimizer-strategy=None -c $C/hip/pqh_assign.hip -o $D/pqh_assign.o &&
    objs=$(ls $O/*.o | grep -v '/pqh_assign.o$') &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpqh.so $objs $D/pqh_assign.o -lpthread &&
    rm $D/pqh_assign.o ) &
done
wait
