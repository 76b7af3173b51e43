set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
bash tools/gpu_sched_ab.sh "--steps,20,--warmup,5;--steps,20,--warmup,5,--hist-on,assign" || exit 1
done
bash tools/gpu_sched_ab.sh "--steps,200,--warmup,20;--steps,200,--warmup,20,--hist-on,assign;--sort,--steps,100,--warmup,10;--sort,--steps,100,--warmup,10,--hist-tune,2x1024;--config,deep,--steps,20,--warmup,5;--config,deep,--steps,20,--warmup,5,--hist-on,assign" || exit 1
