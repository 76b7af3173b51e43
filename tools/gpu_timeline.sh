# Stage timeline of a 20-step bench run (--timeline, every stage's events inside the timed
# steps) plus the drain-builder variants at the driver's 20/5:  bash tools/gpu_timeline.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/tl; mkdir -p $O
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timeline --stage-events timed > $O/tl.log 2> $O/tl.err || { tail $O/tl.err; exit 1; }
grep -o '"value": [0-9.]*' $O/tl.log
for r in 1 2; do
 for dt in default wave lane grp; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --drain-trees $dt > $O/d_$dt.$r.log 2>&1 || { tail $O/d_$dt.$r.log; exit 1; }
  echo "drain=$dt $(grep -o '"value": [0-9.]*' $O/d_$dt.$r.log)"
 done
done
