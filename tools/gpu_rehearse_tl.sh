# Where the multi-rank pipeline's per-rank gap goes (one rank over RCCL, SIFT 1M, 20 steps):
# the stage timeline of the rehearsal and of the one-rank pipeline, then a kernel trace of the
# rehearsal (bench.py started directly, its rendezvous from the environment, no launcher)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/rtl; mkdir -p $O
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
timeout -k 10 200 python bench.py --dist-rehearse --steps 20 --warmup 5 --no-cpu-baseline --timeline --stage-events timed > $O/dist.log 2> $O/dist.err || { tail $O/dist.err; exit 1; }
grep -o '"value": [0-9.]*' $O/dist.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timeline --stage-events timed > $O/one.log 2> $O/one.err || { tail $O/one.err; exit 1; }
grep -o '"value": [0-9.]*' $O/one.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o dist --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --dist-rehearse --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
grep -o '"value": [0-9.]*' $GRAFT_REPO_ROOT/$O/prof.log
