#!/bin/bash
# Diagnostic A/B builds of libpqh with extra compile flags on one source file:
#   bash tools/build_flag_variants.sh <source.hip> "name=-DFLAG=1 -DOTHER=2" ...
#        -> pq_huffman_amd/lib/variants/<name>/libpqh.so  (PQH_LIB=... selects one)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/pq_huffman_amd/csrc; O=$R/pq_huffman_amd/lib/obj
SRC=$1; shift; base=$(basename "$SRC" .hip)
extra=""; [ "$base" = pqh_assign ] && extra="-mllvm -amdgpu-atomic-optimizer-strategy=None"
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}; D=$R/pq_huffman_amd/lib/variants/$name
  rm -rf "$D"; mkdir -p "$D"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$R/include \
     $flags $extra -c $C/hip/$base.hip -o $D/$base.o &
done
wait
for spec in "$@"; do
  D=$R/pq_huffman_amd/lib/variants/${spec%%=*}
  objs=$(ls $O/*.o | grep -v "/$base.o\$")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpqh.so $objs $D/$base.o -lpthread
  rm $D/$base.o
done
