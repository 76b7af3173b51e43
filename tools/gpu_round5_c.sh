set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r9
timeout -k 10 600 python -u -m pytest tests/test_gpu_parts.py tests/test_gpu_lds_poison.py tests/test_gpu_bench_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r9/tests.log 2>&1 || { tail -30 gpurun_out/r9/tests.log; exit 1; }
tail -1 gpurun_out/r9/tests.log
for i in 1 2; do
bash tools/gpu_sched_ab.sh "--steps,200,--warmup,20;--steps,200,--warmup,20,--hist-on,lanes,--hist-tune,4x256;--steps,200,--warmup,20,--hist-on,lanes,--hist-tune,2x256;--steps,200,--warmup,20,--hist-on,lanes,--hist-tune,8x256;--steps,20,--warmup,5;--steps,20,--warmup,5,--hist-on,lanes;--config,deep,--steps,100,--warmup,10;--config,deep,--steps,100,--warmup,10,--hist-on,lanes;--config,deep,--steps,100,--warmup,10,--hist-on,lanes,--hist-tune,8x256" || exit 1
done
bash tools/gpu_sched_ab.sh "--vectors,125000000,--steps,3,--warmup,1;--vectors,125000000,--steps,3,--warmup,1,--hist-on,lanes" || exit 1
