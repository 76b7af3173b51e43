set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/g11; mkdir -p $O
export TMPDIR=/tmp; cd /tmp
for f in wave thread; do
  PQH_HIST_IMPL=$f timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt_$f -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_hist.py deep > $O/kt_$f.log 2>&1 || { tail $O/kt_$f.log; exit 1; }
  PQH_HIST_IMPL=$f timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $O/pmc_$f -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_hist.py deep > $O/pmc_$f.log 2>&1 || { tail $O/pmc_$f.log; exit 1; }
done
echo ok
