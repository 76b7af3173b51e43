set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6/ms
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6/ms/tests.log 2>&1 || { tail -30 gpurun_out/r6/ms/tests.log; exit 1; }
tail -1 gpurun_out/r6/ms/tests.log
bash tools/gpu_lib_ab.sh "--steps 20 --warmup 5" 3 oldmemset && bash tools/gpu_lib_ab.sh "--steps 200 --warmup 10" 2 oldmemset
