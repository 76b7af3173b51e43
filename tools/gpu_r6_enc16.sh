# Encoder change check: the encode / decode parity tests, encode alone, then the bench (SIFT, Deep)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/enc16; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_huffman.py tests/test_gpu_parts.py tests/test_gpu_lds_poison.py "tests/test_gpu_fullsize.py::test_bench_parts_path_sift1m_all_rows" "tests/test_gpu_fullsize.py::test_bench_parts_path_deep1m_all_rows" "tests/test_gpu_fullsize.py::test_encode_segmented_scan_5m_rows" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in sift deep; do
  timeout -k 10 300 python tools/bench_encdec.py --config $c --rows 1000000 --enc-impl 1 --reps 20 > $O/ed_$c.log 2>&1 || { tail $O/ed_$c.log; exit 1; }
  tail -1 $O/ed_$c.log
done
for r in 1 2; do
  for c in sift deep; do
    timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$c.$r.log 2>&1 || { tail $O/b_$c.$r.log; exit 1; }
    echo "$c r$r $(grep -o '"value": [0-9.]*' $O/b_$c.$r.log)"
  done
done
