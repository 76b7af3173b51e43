# list counters, then SQ passes over the assign-only diagnostic
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp; cd /tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 120 python3 $R/tools/bench_assign.py 20 > $R/gpurun_out/assign_plain.log 2>&1 || exit 1
bash $R/tools/pmc_assign.sh probe \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
