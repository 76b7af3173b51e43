# Assignment variants alone at several grid occupancies (PQH_ASSIGN_WGS_PER_CU), SIFT:
#   bash tools/gpu_assign_occ.sh <variant> ...
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/assign_occ; mkdir -p $O
for v in default "$@"; do
  L=pq_huffman_amd/lib/libpqh.so; [ $v != default ] && L=pq_huffman_amd/lib/variants/$v/libpqh.so
  for w in 2 2.5 3 4; do
    PQH_ASSIGN_WGS_PER_CU=$w PQH_LIB=$L timeout -k 10 120 python tools/bench_assign.py 50 sift > $O/$v.$w.log 2>&1 || { tail $O/$v.$w.log; exit 1; }
    echo "$v wgs=$w $(tail -1 $O/$v.$w.log)"
  done
done
