# round-5 profiles, part 1: SIFT (headline), Deep, K = 4,096 (profiles/collect.sh each)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/collect.sh r5_sift && bash profiles/collect.sh r5_deep --config deep && \
bash profiles/collect.sh r5_k4096 --config k4096 --steps 100 --warmup 10
