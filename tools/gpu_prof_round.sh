# The round's profiles (profiles/collect.sh per configuration) + the assignment's SQ counters:
#   bash tools/gpu_prof_round.sh <round tag, e.g. r4> [125m]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:?tag}
bash profiles/collect.sh ${T}_sift && bash profiles/collect.sh ${T}_deep --config deep && \
bash profiles/collect.sh ${T}_k4096 --config k4096 --steps 100 --warmup 10 && \
bash profiles/collect.sh ${T}_sift_sort --sort && \
bash tools/assign_pmc_ab.sh ${T}_final sift pq || exit 1
if [ "$2" = 125m ]; then bash profiles/collect.sh ${T}_125m --vectors 125000000 --steps 3 --warmup 1 || exit 1; fi
