#!/bin/bash
# Diagnostic A/B builds of libpqh with the assignment kernel's compile-time knobs:
#   bash tools/build_variants.sh "WPG OCC NB DEFER" ...
#        -> pq_huffman_amd/lib/variants/<w>_<o>_<p>_<d>/libpqh.so
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/pq_huffman_amd/csrc; O=$R/pq_huffman_amd/lib/obj
rm -rf $R/pq_huffman_amd/lib/variants
for cfg in "$@"; do
  set -- $cfg; D=$R/pq_huffman_amd/lib/variants/$1_$2_$3_$4; mkdir -p $D
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$R/include \
     -DPQH_ASSIGN_WPG=$1 -DPQH_ASSIGN_OCC=$2 -DPQH_ASSIGN_NB=$3 -DPQH_ASSIGN_DEFER=$4 ${EXTRA:-} \
     -mllvm -amdgpu-atomic-optimizer-strategy=None -c $C/hip/pqh_assign.hip -o $D/pqh_assign.o &
done
wait
for D in $R/pq_huffman_amd/lib/variants/*; do
  objs=$(ls $O/*.o | grep -v '/pqh_assign.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpqh.so $objs $D/pqh_assign.o -lpthread
  rm $D/pqh_assign.o
done
