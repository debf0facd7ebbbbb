#!/bin/bash
# One-GPU rehearsal of the driver's multi-GPU bench: 2 ranks on cuda:0 over gloo (RCCL needs one
# device per rank).  Numbers are meaningless (gloo stages through host memory); the point is that
# the default workload runs end to end at N = 2 and prints ONE line with the nested "sharded" record.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export GRACE_BENCH_ONE_DEVICE=1 GRACE_BENCH_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/w2.log 2>&1 || { tail -30 gpurun_out/w2.log; exit 1; }
grep '^{' gpurun_out/w2.log
