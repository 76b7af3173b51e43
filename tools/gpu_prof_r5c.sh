# round-5 profiles, part 3 (after the 256-thread scan): SIFT and the 125M-row shard
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/collect.sh r5_final_sift && \
bash profiles/collect.sh r5_final_125m --vectors 125000000 --steps 3 --warmup 1
