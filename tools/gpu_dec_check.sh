# Decoder change check: the decode parity tests, decode alone (SIFT, Deep) and the bench
# (SIFT, Deep at 200 steps; SIFT at 20) for the in-tree library against lib/variants/<v>:
#   bash tools/gpu_dec_check.sh <variant>
set -o pipefail
V=$1
cd $GRAFT_REPO_ROOT; O=gpurun_out/dec_check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_huffman.py tests/test_gpu_parts.py tests/test_gpu_lds_poison.py "tests/test_gpu_fullsize.py::test_bench_parts_path_sift1m_all_rows" "tests/test_gpu_fullsize.py::test_bench_parts_path_deep1m_all_rows" "tests/test_gpu_fullsize.py::test_bench_path_k4096_1m_all_rows" "tests/test_gpu_fullsize.py::test_encode_segmented_scan_5m_rows" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in default $V; do
    L=pq_huffman_amd/lib/libpqh.so; [ $v != default ] && L=pq_huffman_amd/lib/variants/$v/libpqh.so
    for c in sift deep; do
      PQH_LIB=$L timeout -k 10 300 python tools/bench_encdec.py --config $c --reps 20 > $O/ed_${v}_$c.$r.log 2>&1 || { tail $O/ed_${v}_$c.$r.log; exit 1; }
      echo "$v $(tail -1 $O/ed_${v}_$c.$r.log)"
    done
    for spec in "sift 200" "deep 200" "sift 20"; do
      set -- $spec
      PQH_LIB=$L timeout -k 10 200 python bench.py --config $1 --steps $2 --warmup 5 --no-cpu-baseline > $O/b_${v}_$1_$2.$r.log 2>&1 || { tail $O/b_${v}_$1_$2.$r.log; exit 1; }
      echo "$v $1 K=$2 $(grep -o '"value": [0-9.]*' $O/b_${v}_$1_$2.$r.log) $(grep -o '"decode": [0-9.]*' $O/b_${v}_$1_$2.$r.log)"
    done
  done
done
