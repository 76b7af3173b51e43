# round-4 configs[2] per-rank shard (125M rows) profiles, rows and part-major code layouts
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/collect.sh r4_125m --vectors 125000000 --steps 3 --warmup 1 && \
bash profiles/collect.sh r4_125m_parts --vectors 125000000 --steps 3 --warmup 1 --code-layout parts
