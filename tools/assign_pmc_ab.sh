#!/bin/bash
# SQ instruction mix of the assignment kernel for each PQH_ASSIGN_IMPL (diagnostic):
#   bash tools/assign_pmc_ab.sh <tag> <config> <impl> [impl ...]
# one rocprofv3 --pmc pass per counter group and implementation, over tools/bench_assign.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; CFG=$2; shift 2
export TMPDIR=/tmp; cd /tmp
for impl in "$@"; do
  i=0
  for CTR in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"; do
    PQH_ASSIGN_IMPL=$impl timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$R/gpurun_out/pmc_assign_${TAG}_${impl}_$i" -o pmc \
        --output-format csv -- python3 "$R/tools/bench_assign.py" 5 "$CFG" > "$R/gpurun_out/pmc_assign_${TAG}_${impl}_$i.log" 2>&1 \
        || { tail "$R/gpurun_out/pmc_assign_${TAG}_${impl}_$i.log"; exit 1; }
    i=$((i+1))
  done
done
echo pmc done
