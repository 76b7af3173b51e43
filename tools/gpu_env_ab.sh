# Bench lines under environment variants: bash tools/gpu_env_ab.sh "<bench args>" "<ENV=.. ENV=..>|-" ...
# ("-" = no extra environment); each variant once, in order
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/envab; mkdir -p $OUT
A=$1; shift
i=0
for e in "$@"; do
  i=$((i+1)); [ "$e" = "-" ] && e=""
  timeout -k 10 300 env $e python bench.py $A --no-cpu-baseline > $OUT/r$i.log 2>&1 || { tail $OUT/r$i.log; exit 1; }
  echo "[$e] $(grep -o '"value": [0-9.]*' $OUT/r$i.log) $(grep -o '"stages_ms": {[^}]*}' $OUT/r$i.log)"
done
