#!/bin/bash
# One-GPU rehearsal of the driver's multi-GPU bench at N ranks (default 2 and 4) on cuda:0 over
# gloo (RCCL needs one device per rank).  Numbers are meaningless (gloo stages through host
# memory); the point is that the default workload runs end to end and prints ONE line with the
# nested "sharded" record.  usage: tools/wn_rehearsal.sh [N ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export GRACE_BENCH_ONE_DEVICE=1 GRACE_BENCH_BACKEND=gloo
for N in ${@:-2 4}; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 > gpurun_out/w$N.log 2>&1 \
    || { tail -30 gpurun_out/w$N.log; exit 1; }
  grep '^{' gpurun_out/w$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($N, d['n_gpus'], d['ms_per_step'], d['sharded']['ms_per_step'], d['sharded']['config']['shard'])"
done
