# Assignment change check: the assignment's parity tests, then the kernel alone and the bench
# (SIFT, Deep) for the in-tree library against lib/variants/<v>, interleaved, two rounds:
#   bash tools/gpu_assign_ab.sh <variant>
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/assign_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_configs.py "tests/test_gpu_fullsize.py::test_bench_parts_path_sift1m_all_rows" "tests/test_gpu_fullsize.py::test_bench_parts_path_deep1m_all_rows" "tests/test_gpu_fullsize.py::test_bench_path_k4096_1m_all_rows" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in default $1; do
    L=pq_huffman_amd/lib/libpqh.so; [ $v != default ] && L=pq_huffman_amd/lib/variants/$v/libpqh.so
    for c in sift deep; do
      PQH_LIB=$L timeout -k 10 120 python tools/bench_assign.py 50 $c > $O/ba_${v}_$c.$r.log 2>&1 || { tail $O/ba_${v}_$c.$r.log; exit 1; }
      echo "$v $(tail -1 $O/ba_${v}_$c.$r.log)"
    done
    for K in 20 200; do
      PQH_LIB=$L timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline > $O/b_$v.$K.$r.log 2>&1 || { tail $O/b_$v.$K.$r.log; exit 1; }
      echo "$v K=$K $(grep -o '"value": [0-9.]*' $O/b_$v.$K.$r.log)"
    done
  done
done
