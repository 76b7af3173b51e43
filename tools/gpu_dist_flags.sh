# One-rank RCCL rehearsal (bench.py --dist-rehearse) flag variants at 20 steps, two rounds:
#   bash tools/gpu_dist_flags.sh "label:flags" ...
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/distflags; mkdir -p $O
for r in 1 2; do
  for spec in "$@"; do
    L=${spec%%:*}; F=${spec#*:}
    timeout -k 10 200 python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nnodes=1 --nproc-per-node=1 bench.py --dist-rehearse --steps ${K:-20} --warmup 5 --no-cpu-baseline $F > $O/$L.$r.log 2>&1 || { tail -5 $O/$L.$r.log; exit 1; }
    echo "$L r$r $(grep -o '"value": [0-9.]*' $O/$L.$r.log) $(grep -o '"decode": [0-9.]*' $O/$L.$r.log)"
  done
done
