set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_enc; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $OUT -o pmc --output-format csv -- python3 $R/tools/bench_encode.py > $OUT/log 2>&1
