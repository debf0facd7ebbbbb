"""Headline benchmark: grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket.

Workload (BASELINE.json configs[1]): one ``Allgather(TopKCompressor(0.01), ResidualMemory(), N)
.step(g, name)`` per step on a 256 MiB fp32 gradient bucket already resident in HBM:
compensate (t = r + g) -> top-k 1 % -> residual update -> payload exchange -> decode+aggregate.
value = N * 4n bytes / step time (whole job), n = 67,108,864.

At N > 1 every rank runs its own bucket (data-parallel replicas of the reference's Allgather
semantics); the fixed-size payloads (k f32 values + k i32 indices) move with one RCCL
all_gather_into_tensor per step and are decoded + aggregated in rank order on every rank.

Launch: ``python bench.py`` (N=1) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--numel", type=int, default=64 * 1024 * 1024)
    ap.add_argument("--buffers", type=int, default=3, help="distinct buckets rotated (defeats MALL reuse)")
    ap.add_argument("--cpu-baseline-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 needs torch.distributed.run with N processes")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory

    n = args.numel
    k = ops.ratio_k(n, args.ratio)
    comm = Allgather(TopKCompressor(args.ratio), ResidualMemory(), world)
    gen = torch.Generator(device=dev)
    grads = []
    for j in range(args.buffers):
        gen.manual_seed(1000 * rank + j + 1)
        grads.append(torch.randn(n, device=dev, generator=gen))
    names = [f"bucket{j}" for j in range(args.buffers)]

    def step(i):
        j = i % args.buffers
        return comm.step(grads[j], names[j])

    # warm-up (first step per name has no residual; run every name at least once)
    for i in range(max(args.warmup, args.buffers)):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    ops.timer_enable(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    main_ms, launches = ops.timer_collect()
    ops.timer_enable(False)
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed / args.steps * 1e3
    value = world * 4.0 * n * args.steps / elapsed / 1e9

    # roofline of the dominant kernel (topk_main), timed with HIP events on its own stream
    main_avg_ms = main_ms / max(launches, 1)
    bytes_per_elem = 16 if world == 1 else 12          # g, r read; r' (+ dense out at W=1) written
    main_bytes = bytes_per_elem * n
    achieved = main_bytes / (main_avg_ms * 1e-3) / 1e9
    step_bytes = 16 * n + 16 * k if world == 1 else None
    roofline = {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
        "kernel": "topk_main", "kernel_avg_us": round(main_avg_ms * 1e3, 2),
        "algorithmic_bytes_per_launch": main_bytes,
    }
    if step_bytes:
        roofline["step_frac"] = round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    prof = os.path.join(ROOT, "profiles", "pmc_topk_main.json")
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                pmc = json.load(f)
            if pmc.get("numel") == n and pmc.get("world") == world:
                roofline["traffic"] = pmc["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            pass

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_steps > 0:
        cpu = cpu_baseline(n, args.ratio, args.cpu_baseline_steps)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (torch.randn buckets, 3 rotated per rank)",
            "config": {"workload": "Allgather(TopK 1% , ResidualMemory).step on a 256 MiB fp32 bucket "
                                   "(BASELINE configs[1])",
                       "numel": n, "k": k, "parallelism": f"dp{world} replicas, RCCL allgather of payloads"},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(n, ratio, steps):
    """The oracle's top-k + residual step on the host cores over the same bucket size."""
    import numpy as np
    from oracle import grace_oracle as O
    threads = torch.get_num_threads()
    rng = np.random.default_rng(0)
    g = rng.standard_normal(n, dtype=np.float32)
    r = (0.1 * rng.standard_normal(n, dtype=np.float32)).astype(np.float32)
    O.topk_residual_step(g[: 1 << 20], r[: 1 << 20], ratio)     # warm
    t0 = time.perf_counter()
    for _ in range(steps):
        _, _, _, r, _ = O.topk_residual_step(g, r, ratio)
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(4.0 * n / dt / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{steps} full 256 MiB top-k 1% + residual steps of oracle/grace_oracle.py "
                      f"(numpy partition + torch CPU ops), {dt * 1e3:.0f} ms/step"}


if __name__ == "__main__":
    main()
