# A round's profiles: profiles/collect.sh per configuration (bench line, kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes):  bash tools/gpu_prof_round.sh <tag prefix, e.g. r6_final> <set>
#   set a: sift deep sift_sort;  set b: k4096 + the assignment's SQ counters;  set c: 125m
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:?tag}
case $2 in
  a) bash profiles/collect.sh ${T}_sift && bash profiles/collect.sh ${T}_deep --config deep && \
     bash profiles/collect.sh ${T}_sift_sort --sort ;;
  b) bash profiles/collect.sh ${T}_k4096 --config k4096 --steps 100 --warmup 10 && \
     bash tools/assign_pmc_ab.sh ${T} sift pq ;;
  c) bash profiles/collect.sh ${T}_125m --vectors 125000000 --steps 6 --warmup 1 ;;
esac
