# Full GPU suite, then the default bench (200 steps, and the driver's 20/5) twice, then an
# optional SQ-mix pass (tools/bench_sq_mix.sh <tag>):  bash tools/gpu_check.sh [sqmix tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/check; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for K in 200 20; do
    W=10; [ $K = 20 ] && W=5
    timeout -k 10 300 python bench.py --steps $K --warmup $W --no-cpu-baseline > $OUT/b$K.$i.log 2>&1 || { tail $OUT/b$K.$i.log; exit 1; }
    echo "K=$K $(grep -o '"value": [0-9.]*' $OUT/b$K.$i.log) $(grep -o '"stages_ms": {[^}]*}' $OUT/b$K.$i.log)"
  done
done
if [ -n "$1" ]; then bash tools/bench_sq_mix.sh "$1" || exit 1; fi
