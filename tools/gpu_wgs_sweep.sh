# Assignment grid occupancy sweep in the bench (--assign-wgs-per-cu), two rounds:
#   bash tools/gpu_wgs_sweep.sh "<bench args>" <wgs>...
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/wgs; mkdir -p $OUT
A=$1; shift
for i in 1 2; do
  for w in "$@"; do
    timeout -k 10 300 python bench.py $A --assign-wgs-per-cu $w --no-cpu-baseline > $OUT/w$w.$i.log 2>&1 || { tail $OUT/w$w.$i.log; exit 1; }
    echo "[$A] wgs $w $(grep -o '"value": [0-9.]*' $OUT/w$w.$i.log) $(grep -o '"stages_ms": {[^}]*}' $OUT/w$w.$i.log)"
  done
done
