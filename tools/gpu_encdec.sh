# Encode / decode alone (tools/bench_encdec.py) at 1M and 125M rows, both encoders
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/encdec; mkdir -p $O
for spec in "sift 1000000 1" "sift 1000000 2" "deep 1000000 1" "deep 1000000 2" "sift 125000000 1" "sift 125000000 2"; do
  set -- $spec
  timeout -k 10 300 python tools/bench_encdec.py --config $1 --rows $2 --enc-impl $3 --reps ${REPS:-10} > $O/$1_$2_$3.log 2>&1 || { tail $O/$1_$2_$3.log; exit 1; }
  tail -1 $O/$1_$2_$3.log
done
