set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export GRACE_BENCH_ONE_DEVICE=1 GRACE_BENCH_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/w2.log 2>&1 || { tail -30 gpurun_out/w2.log; exit 1; }
grep '^{' gpurun_out/w2.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --workload topk_sharded > gpurun_out/w2s.log 2>&1 || { tail -30 gpurun_out/w2s.log; exit 1; }
grep '^{' gpurun_out/w2s.log
