# multi-rank plumbing of the bench on the box's one GPU: 2 ranks, host-staged exchange (RCCL
# refuses two ranks on one GPU), C3 and C5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/mr; mkdir -p $O
for cfg in c3 c5; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --comm host --config $cfg \
    > $O/bench_${cfg}_2rank_host.log 2>&1 || { tail -20 $O/bench_${cfg}_2rank_host.log; exit 1; }
  grep '^{' $O/bench_${cfg}_2rank_host.log | cut -c1-400
done
