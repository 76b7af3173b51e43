# Bench A/B of the in-tree library against lib/variants/<v> (PQH_LIB), interleaved on one box:
#   bash tools/gpu_lib_ab.sh "<bench args>" <rounds> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/libab; mkdir -p $OUT
A=$1; R=$2; shift 2
for i in $(seq 1 $R); do
  for v in in-tree "$@"; do
    L=""; [ "$v" != in-tree ] && L=$GRAFT_REPO_ROOT/pq_huffman_amd/lib/variants/$v/libpqh.so
    env ${L:+PQH_LIB=$L} timeout -k 10 300 python bench.py $A --no-cpu-baseline > $OUT/$v.$i.log 2>&1 || { tail $OUT/$v.$i.log; exit 1; }
    echo "$v $(grep -o '"value": [0-9.]*' $OUT/$v.$i.log) $(grep -o '"stages_ms": {[^}]*}' $OUT/$v.$i.log)"
  done
done
