set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r8
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_pq.py "tests/test_gpu_fullsize.py::test_bench_path_k4096_1m_all_rows" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r8/tests.log 2>&1 || { tail -30 gpurun_out/r8/tests.log; exit 1; }
tail -1 gpurun_out/r8/tests.log
timeout -k 10 300 python tools/bench_assign.py 20 k4096 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
bash tools/gpu_sched_ab.sh "--config,k4096,--steps,30,--warmup,5;--config,k4096,--steps,30,--warmup,5,--pair-tables,--lanes,2,--elanes,1" || exit 1
for i in 1 2; do
bash tools/gpu_env_ab.sh "--config deep --steps 100 --warmup 10" - PQH_HIST_BLOCK=256 || exit 1
bash tools/gpu_env_ab.sh "--steps 200 --warmup 20" - || exit 1
bash tools/gpu_env_ab.sh "--steps 200 --warmup 20 --hist-on lanes" "PQH_HIST_SPLIT=4 PQH_HIST_BLOCK=256" || exit 1
done
