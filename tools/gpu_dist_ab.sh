# One-rank RCCL rehearsal of the multi-rank pipeline against the one-rank pipeline:
#   bash tools/gpu_dist_ab.sh [steps ...]
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/dist; mkdir -p $O
for r in 1 2; do
  for K in ${@:-20}; do
    timeout -k 10 200 python bench.py --steps $K --warmup 5 --no-cpu-baseline > $O/one.$K.$r.log 2>&1 || { tail $O/one.$K.$r.log; exit 1; }
    echo "one K=$K $(grep -o '"value": [0-9.]*' $O/one.$K.$r.log)"
    timeout -k 10 200 python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nnodes=1 --nproc-per-node=1 bench.py --dist-rehearse --steps $K --warmup 5 --no-cpu-baseline ${DFLAGS:-} > $O/reh.$K.$r.log 2>&1 || { tail $O/reh.$K.$r.log; exit 1; }
    echo "rehearse K=$K $(grep -o '"value": [0-9.]*' $O/reh.$K.$r.log) $(grep -o '"stages_ms": {[^}]*}' $O/reh.$K.$r.log)"
  done
done
timeout -k 10 200 python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nnodes=1 --nproc-per-node=1 bench.py --dist-rehearse --steps 20 --warmup 5 --no-cpu-baseline --timeline --stage-events timed ${DFLAGS:-} > $O/tl.log 2> $O/tl.err || { tail $O/tl.err; exit 1; }
