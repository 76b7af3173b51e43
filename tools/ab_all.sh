set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pq.log 2>&1 || { tail -30 gpurun_out/gpu_pq.log; exit 1; }
tail -1 gpurun_out/gpu_pq.log
for i in 1 2; do
  echo "== in-tree"; BENCH_ASSIGN_EXACT=0 timeout -k 10 200 python tools/bench_assign.py 50 all 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== base"; PQH_LIB=$R/pq_huffman_amd/lib/variants/base/libpqh.so BENCH_ASSIGN_EXACT=0 timeout -k 10 200 python tools/bench_assign.py 50 all 2>&1 | grep -v amdgpu.ids || exit 1
done
