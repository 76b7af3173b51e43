# Stage timeline of the 125M-row shard bench (configs[2] per rank): bash tools/gpu_timeline_125m.sh [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/tl125; mkdir -p $O
S=${1:-3}
timeout -k 10 400 python bench.py --vectors 125000000 --steps $S --warmup 1 --no-cpu-baseline --timeline --stage-events timed > $O/tl$S.log 2> $O/tl$S.err || { tail $O/tl$S.err; exit 1; }
grep -o '"value": [0-9.]*' $O/tl$S.log
grep "^TL" $O/tl$S.err
