set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r7
timeout -k 10 120 ./tools/micro/lds_peek64 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_pq.py tests/test_gpu_parts.py tests/test_gpu_configs.py tests/test_gpu_huffman.py tests/test_gpu_lds_poison.py "tests/test_gpu_fullsize.py::test_bench_path_k4096_1m_all_rows" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r7/tests.log 2>&1 || { tail -30 gpurun_out/r7/tests.log; exit 1; }
tail -1 gpurun_out/r7/tests.log
timeout -k 10 300 python tools/bench_assign.py 20 k4096 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/gpu_sched_ab.sh "--config,k4096,--steps,30,--warmup,5;--config,k4096,--steps,30,--warmup,5,--pair-tables,--lanes,2,--elanes,1;--config,k4096,--steps,30,--warmup,5,--lanes,2,--elanes,1" || exit 1
bash tools/gpu_env_ab.sh "--config deep --steps 100 --warmup 10" - PQH_HIST_SPLIT=4 PQH_HIST_BLOCK=256 "PQH_HIST_SPLIT=4 PQH_HIST_BLOCK=256" || exit 1
bash tools/gpu_env_ab.sh "--steps 200 --warmup 20" - PQH_HIST_SPLIT=4 || exit 1
bash tools/gpu_lib_ab.sh "--steps 200 --warmup 20" 2 xnt || exit 1
# the 2-rank rehearsal (gloo, both ranks on this GPU) beside an N = 1 run, per-rank Mvec/s
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --dist-backend gloo --one-device --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r7/ranks2.log 2>&1 || { tail -20 gpurun_out/r7/ranks2.log; exit 1; }
echo "2 ranks on one GPU: $(grep -o '"value": [0-9.]*' gpurun_out/r7/ranks2.log) $(grep -o '"code_layout": "[a-z]*"' gpurun_out/r7/ranks2.log)"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r7/ranks1.log 2>&1 || exit 1
echo "1 rank: $(grep -o '"value": [0-9.]*' gpurun_out/r7/ranks1.log)"
bash tools/gpu_env_ab.sh "--steps 200 --warmup 20 --hist-on lanes" "PQH_HIST_SPLIT=8 PQH_HIST_BLOCK=256" "PQH_HIST_SPLIT=4 PQH_HIST_BLOCK=256" || exit 1
