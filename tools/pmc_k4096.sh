#!/bin/bash
# PMC passes over the K=4096 assignment (diagnostic) -> gpurun_out/pmc_k4096_<i>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp BENCH_ASSIGN_EXACT=0; cd /tmp
i=0
for CTR in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"; do
  OUT=$R/gpurun_out/pmc_k4096/pmc_$i; mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT" -o pmc --output-format csv \
      -- python3 "$R/tools/bench_assign.py" 3 k4096 > "$OUT/log" 2>&1 || { tail "$OUT/log"; exit 1; }
  i=$((i+1))
done
echo done
