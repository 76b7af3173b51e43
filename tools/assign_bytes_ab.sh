# HBM bytes and time of the assignment alone (tools/bench_assign.py), row-major vs part-major
# codes, for the in-tree library and each lib/variants/<v> given
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp; cd /tmp
run() {   # $1 label, $2 parts flag, $3 lib (or empty)
  for CTR in FETCH_SIZE WRITE_SIZE; do
    env ${3:+PQH_LIB=$3} BENCH_ASSIGN_PARTS=$2 timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$R/gpurun_out/bytes_$1_$CTR" -o pmc --output-format csv \
        -- python3 "$R/tools/bench_assign.py" 5 > "$R/gpurun_out/bytes_$1_$CTR.log" 2>&1 || { tail "$R/gpurun_out/bytes_$1_$CTR.log"; exit 1; }
    python3 - "$R/gpurun_out/bytes_$1_$CTR/pmc_counter_collection.csv" $1 $CTR <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "pq_assign_mfma" in r["Kernel_Name"]]
print(sys.argv[2], sys.argv[3], "KB per launch", [round(x) for x in v[-3:]])
PY
  done
  env ${3:+PQH_LIB=$3} BENCH_ASSIGN_PARTS=$2 timeout -k 10 120 python3 "$R/tools/bench_assign.py" 50 2>&1 | grep -v amdgpu.ids | sed "s/^/$1 /"
}
run rows 0 "" && run parts 1 ""
for v in "$@"; do run "parts_$v" 1 "$R/pq_huffman_amd/lib/variants/$v/libpqh.so" || exit 1; done
