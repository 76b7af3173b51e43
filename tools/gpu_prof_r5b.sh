# round-5 profiles, part 2: sort mode, the 125M-row shard, the assignment's SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/collect.sh r5_sift_sort --sort && \
bash tools/assign_pmc_ab.sh r5_final sift pq && \
bash profiles/collect.sh r5_125m --vectors 125000000 --steps 3 --warmup 1
