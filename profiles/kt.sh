set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/kt_$1; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/log 2>&1
