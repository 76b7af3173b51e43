#!/bin/bash
# Assignment A/B + evidence on the GPU box (diagnostic):
#   bash tools/assign_ab_prof.sh <tag> [variant ...]
# 1. the GPU PQ parity tests (in-tree library), 2. tools/bench_assign.py for the in-tree
# library and each variant under pq_huffman_amd/lib/variants, 3. rocprofv3 kernel trace of
# the in-tree assignment, 4. PMC passes (SQ instruction mix / busy cycles, HBM bytes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; shift
OUT=$R/gpurun_out/assign_$TAG; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_pq.py" -x -q --timeout 120 \
    --timeout-method thread > "$OUT/gpu_pq.log" 2>&1 || { tail -30 "$OUT/gpu_pq.log"; exit 1; }
tail -1 "$OUT/gpu_pq.log"
for i in 1 2; do
  echo -n "in-tree: "; timeout -k 10 120 python "$R/tools/bench_assign.py" 50 2>&1 | grep -v amdgpu.ids || exit 1
  for v in "$@"; do
    echo -n "$v: "; PQH_LIB=$R/pq_huffman_amd/lib/variants/$v/libpqh.so \
      timeout -k 10 120 python "$R/tools/bench_assign.py" 50 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
export TMPDIR=/tmp; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 "$R/tools/bench_assign.py" 20 > "$OUT/kt.log" 2>&1 || { tail "$OUT/kt.log"; exit 1; }
i=0
for CTR in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT/pmc_$i" -o pmc --output-format csv \
      -- python3 "$R/tools/bench_assign.py" 5 > "$OUT/pmc_$i.log" 2>&1 || { tail "$OUT/pmc_$i.log"; exit 1; }
  i=$((i+1))
done
echo done
