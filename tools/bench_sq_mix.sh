#!/bin/bash
# SQ instruction mix of every kernel in the bench schedule (diagnostic: which side kernel
# takes issue slots from the assignment): two rocprofv3 --pmc passes over a short bench run
#   bash tools/bench_sq_mix.sh <tag> [bench args]   -> gpurun_out/sqmix_<tag>_{0,1}/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; shift
export TMPDIR=/tmp; cd /tmp
i=0
for CTR in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  timeout -s KILL 150 rocprofv3 --pmc $CTR -d "$R/gpurun_out/sqmix_${TAG}_$i" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --steps 10 --warmup 2 --device-warmup-ms 0 --no-cpu-baseline "$@" \
      > "$R/gpurun_out/sqmix_${TAG}_$i.log" 2>&1 || { tail "$R/gpurun_out/sqmix_${TAG}_$i.log"; exit 1; }
  i=$((i+1))
done
echo sqmix done
