# bench.py flag variants at the driver's 20 steps / 5 warmup, three rounds, interleaved:
#   bash tools/gpu_flags.sh "label:flags" ...     (NAME=VALUE words go to the environment)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/r6/flags; mkdir -p $O
for r in 1 2 3; do
  for spec in "$@"; do
    L=${spec%%:*}; F=""; E=()
    for w in ${spec#*:}; do
      if [[ $w =~ ^[A-Z_0-9]+= ]]; then E+=("$w"); else F="$F $w"; fi
    done
    env "${E[@]}" timeout -k 10 200 python bench.py --steps ${K:-20} --warmup 5 --no-cpu-baseline $F > $O/$L.$r.log 2>&1 || { tail -5 $O/$L.$r.log; exit 1; }
    echo "$L r$r $(grep -o '"value": [0-9.]*' $O/$L.$r.log)"
  done
done
