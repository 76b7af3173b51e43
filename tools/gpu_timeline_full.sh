# Every stage's events, the assignment's included, over the timed steps of one-rank runs at
# 20 and 200 steps (unprofiled): where stream A waits.  -> gpurun_out/r6/tlf/
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/tlf; mkdir -p $O
for K in 20 200; do
  timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline --timeline --stage-events timed --assign-event-every 1 > $O/tl$K.log 2> $O/tl$K.err || { tail $O/tl$K.err; exit 1; }
  echo "K=$K $(grep -o '"value": [0-9.]*' $O/tl$K.log)"
done
