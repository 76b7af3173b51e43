# The assignment kernel alone (SIFT, Deep), the in-tree library against lib/variants/<v>,
# interleaved, <rounds> rounds:  bash tools/gpu_assign_alone_ab.sh <rounds> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/assign_alone; mkdir -p $O
R=$1; shift
for r in $(seq 1 $R); do
  for v in default "$@"; do
    L=pq_huffman_amd/lib/libpqh.so; [ $v != default ] && L=pq_huffman_amd/lib/variants/$v/libpqh.so
    for c in sift deep; do
      PQH_LIB=$L timeout -k 10 120 python tools/bench_assign.py 50 $c > $O/${v}_$c.$r.log 2>&1 || { tail $O/${v}_$c.$r.log; exit 1; }
      echo "$v $(tail -1 $O/${v}_$c.$r.log)"
    done
  done
done
