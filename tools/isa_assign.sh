#!/bin/bash
# Diagnostic: gfx950 ISA of pq_assign_mfma<16, 8, uint8> -> /tmp/assign16.s, with its register
# counts and the key-reduction instruction mix (static counts over both lo-pass variants).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$R/include" \
    -mllvm -amdgpu-atomic-optimizer-strategy=None --cuda-device-only -S \
    -o /tmp/assign_all.s "$R/pq_huffman_amd/csrc/hip/pqh_assign.hip"
K=_ZN12_GLOBAL__N_114pq_assign_mfmaILi16ELi8EhEEvPKfxxiPKDv8_DF16b
awk -v k="$K" 'index($0,k)==1 && /: ;/{f=1} f&&/s_endpgm/{print; f=0} f' /tmp/assign_all.s > /tmp/assign16.s
grep -A12 "\.name:.*pq_assign_mfmaILi16ELi8Eh" /tmp/assign_all.s | grep -E "vgpr_count|spill" || true
grep -v "^\s*;" /tmp/assign16.s | awk '{print $1}' | grep -E "^v_(min|med|max|and_or|mfma)" \
    | sort | uniq -c
