# The multi-rank pipeline over RCCL rehearsed with one rank: the 1M-row batch at the driver's
# 20/5 and at 200 steps, and configs[2]'s 125M-row per-rank shard -> gpurun_out/r6/rehearse/
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/rehearse; mkdir -p $O
run() {   # label, bench args
  L=$1; shift
  timeout -k 10 400 python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nnodes=1 --nproc-per-node=1 bench.py --dist-rehearse --no-cpu-baseline "$@" > $O/$L.log 2>&1 || { tail -5 $O/$L.log; exit 1; }
  echo "$L $(grep -o '"value": [0-9.]*' $O/$L.log)"
}
run r20 --steps 20 --warmup 5 && run r200 --steps 200 --warmup 10 && \
run r125m --vectors 125000000 --steps 4 --warmup 1
