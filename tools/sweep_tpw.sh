set -o pipefail
for tpw in 32 16 8; do
  export PQH_TREE_TPW=$tpw
  echo "#### TPW $tpw"
  bash tools/sweep_sched.sh "--depth 3 --chunk 8 --table-cus 256" "--depth 3 --chunk 8 --table-cus 128" "--depth 2 --chunk 8 --table-cus 256" || exit 1
done
