# Assignment-only timing of diagnostic builds (tools/build_assign_variant.sh) against the default:
#   bash tools/gpu_assign_variants.sh <variant> ...
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/diag; mkdir -p $O
for r in 1 2; do
 for v in default "$@"; do
  L=pq_huffman_amd/lib/libpqh.so; [ $v != default ] && L=pq_huffman_amd/lib/variants/$v/libpqh.so
  PQH_LIB=$L timeout -k 10 120 python tools/bench_assign.py 50 ${CFG:-sift} > $O/ba_$v.$r.log 2>&1 || { tail $O/ba_$v.$r.log; exit 1; }
  echo "$v $(tail -1 $O/ba_$v.$r.log)"
 done
done
