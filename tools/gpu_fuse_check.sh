# Fused trees + decode tables: the whole GPU suite, then the bench with and without the fusion
# (--split-tables), interleaved, 20 and 100 steps, two rounds each (tools/gpu_benchab.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6/fuse
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6/fuse/tests.log 2>&1 || { tail -30 gpurun_out/r6/fuse/tests.log; exit 1; }
tail -1 gpurun_out/r6/fuse/tests.log
bash tools/gpu_benchab.sh "fused:--fuse-tables" "split:"
