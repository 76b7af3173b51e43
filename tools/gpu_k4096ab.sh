# K = 4096 assignment A/B: the in-tree build and lib/variants/<v> (tools/bench_assign.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/k4096ab; mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "4096" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
for i in 1 2; do
  BENCH_ASSIGN_EXACT=0 timeout -k 10 200 python tools/bench_assign.py 10 k4096 2>&1 | grep -v amdgpu.ids | sed 's/^/in-tree /' || exit 1
  for v in "$@"; do
    PQH_LIB=$GRAFT_REPO_ROOT/pq_huffman_amd/lib/variants/$v/libpqh.so BENCH_ASSIGN_EXACT=0 timeout -k 10 200 python tools/bench_assign.py 10 k4096 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
  done
done
