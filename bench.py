"""Headline benchmark: grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket.

Default workload (BASELINE.json configs[1]): one ``Allgather(TopKCompressor(0.01),
ResidualMemory(), N).step(g, name)`` per step on a 256 MiB fp32 gradient bucket already resident in
HBM: compensate (t = r + g) -> top-k 1 % -> residual update -> payload exchange -> decode +
aggregate.  value = N * 4n bytes / step time (whole job), n = 67,108,864.

At N > 1 every rank runs its own bucket (data-parallel replicas, the reference's Allgather
semantics); the fixed-size payloads (k f32 values + k i32 indices) move with one RCCL
all_gather_into_tensor per step and are decoded + aggregated in rank order on every rank.

Secondary workloads (``--workload``; same JSON schema, reported in DESIGN.md, not the headline):
  sign       signSGD Allgather step, 4 MiB fp32 (configs[0])
  sign256    signSGD Allgather step, 256 MiB fp32
  qsgd       QSGD(127, 128) compress + decompress over the 161-tensor ResNet-50 set, one
             segmented launch per stage (configs[2])
  terngrad   TernGrad, same set (configs[2])
  topk_nomem top-k 1 % without memory, Allgather(TopK, NoneMemory).step on the 256 MiB bucket
             (8n + 16k algorithmic bytes); world 1 is one streaming pass
  topk_e2e   the headline step with the bucket arriving from pinned host memory (H2D) and the
             aggregated dense gradient returned to it (D2H): the PCIe-inclusive rate in DESIGN.md
  topk_sharded  ONE 256 MiB bucket sharded over the N ranks, top-k 0.1 % + residual, exact global
             selection (histogram exchange + boundary lists + payload allgather), replicated dense
             decode (configs[4]); value = 4n / step time (strong scaling: the bucket is fixed)
  ddp_params / ddp_segmented / ddp_bucket  the DDP loopback harness (grace_amd/harness.py) on
             ResNet-50's 161 gradient tensors, top-k 1 % + residual: the per-parameter grc.step loop
             (examples/dist/CIFAR10-dawndist/core.py:204-208), the same per-tensor semantics in one
             launch sequence (SegmentedTopK), and one flat bucket with a single global top-k
  powersgd   PowerSGD rank 4 compress + decompress on a 4096 x 4096 gradient (configs[3])
  dgc        DGC 1 % with momentum-correction memory on the 256 MiB bucket
  sign_bits  signSGD with the 1-bit wire layout, compress + Allgather decode, 256 MiB (8f.4)
  randomk / threshold  RandomK 1 % / Threshold with residual memory on the 256 MiB bucket (8a)

Launch: ``python bench.py`` (N=1) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``.
"""
import argparse
import datetime
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
F32_PEAK_TFLOPS = 157.3        # MI355X dense f32 MFMA peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="topk",
                    choices=["topk", "topk_nomem", "topk_e2e", "topk_sharded", "sign", "sign256", "qsgd", "terngrad", "qsgd_step", "terngrad_step", "powersgd",
                             "natural", "cnat", "fp16", "ddp_params", "ddp_bucket", "ddp_segmented", "dgc",
                             "sign_bits", "randomk", "threshold"])
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--numel", type=int, default=64 * 1024 * 1024)
    ap.add_argument("--buffers", type=int, default=3, help="distinct buckets rotated (defeats MALL reuse)")
    ap.add_argument("--cpu-baseline-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stream", choices=["default", "side"], default="default",
                    help="issue the workload on torch's default stream or on one created stream")
    ap.add_argument("--no-overlap", action="store_true", help="skip the two-stream record of the top-k workload")
    ap.add_argument("--no-sharded", action="store_true",
                    help="at N > 1, skip the nested sharded (configs[4]) measurement of the default workload")
    return ap.parse_args()


def resnet50_shapes():
    """The 161 parameter shapes of torchvision's ResNet-50 (25,557,032 elements)."""
    shapes = [(64, 3, 7, 7), (64,), (64,)]
    inplanes = 64
    for planes, blocks in ((64, 3), (128, 4), (256, 6), (512, 3)):
        for b in range(blocks):
            shapes += [(planes, inplanes, 1, 1), (planes,), (planes,), (planes, planes, 3, 3), (planes,), (planes,),
                       (planes * 4, planes, 1, 1), (planes * 4,), (planes * 4,)]
            if b == 0:
                shapes += [(planes * 4, inplanes, 1, 1), (planes * 4,), (planes * 4,)]
            inplanes = planes * 4
    shapes += [(1000, 2048), (1000,)]
    return shapes


def timed(fn, steps, warmup, world, dev):
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(warmup + i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world == 1:
        raise SystemExit("--gpus N > 1 needs torch.distributed.run with N processes")
    # rehearsal knobs for a one-GPU box (never used by the driver's runs): every rank on cuda:0,
    # gloo instead of RCCL (RCCL needs one device per rank)
    if os.environ.get("GRACE_BENCH_ONE_DEVICE") == "1":
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        backend = os.environ.get("GRACE_BENCH_BACKEND", "nccl")
        # a bounded collective timeout: a rank that never arrives ends the job instead of holding
        # the node until the driver's limit
        tmo = datetime.timedelta(seconds=int(os.environ.get("GRACE_BENCH_PG_TIMEOUT", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    run = {"topk": bench_topk, "topk_nomem": bench_topk_nomem, "topk_e2e": bench_topk_e2e, "topk_sharded": bench_topk_sharded,
           "ddp_params": bench_ddp, "ddp_bucket": bench_ddp, "ddp_segmented": bench_ddp, "sign": bench_sign, "sign256": bench_sign, "qsgd": bench_quant, "qsgd_step": bench_quant, "terngrad_step": bench_quant,
           "terngrad": bench_quant, "powersgd": bench_powersgd, "dgc": bench_dgc, "sign_bits": bench_sign_bits,
           "randomk": bench_sparse, "threshold": bench_sparse, "natural": bench_cast, "cnat": bench_cast,
           "fp16": bench_cast}[args.workload]
    if args.stream == "side":
        with torch.cuda.stream(torch.cuda.Stream(device=dev)):
            line = run(args, world, rank, dev)
    else:
        line = run(args, world, rank, dev)
    if args.workload == "topk" and world > 1 and not args.no_sharded:
        # BASELINE configs[4] (one 256 MiB bucket sharded over the ranks, top-k 0.1 %) rides in the
        # same JSON line, so the driver's 1 -> 8 GPU record covers it next to the DP replicas
        line["sharded"] = nested_sharded(line, args, world, rank, dev)
        # SURVEY §8e's other sharded codecs at the same N: configs[2]'s ResNet-50 set as ONE bucket
        # split over the ranks (sharded TernGrad: one all-gather of unit partials + one of the codes;
        # sharded QSGD: one all-gather of codes + norms), same guard
        for key, codec in (("sharded_terngrad", "terngrad"), ("sharded_qsgd", "qsgd")):
            line[key] = nested_sharded(line, args, world, rank, dev, key=key,
                                       fn=lambda a, w, r, d, c=codec: bench_sharded_codec(a, w, r, d, c))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def nested_sharded(line, args, world, rank, dev, key="sharded", fn=None):
    """The configs[4] record inside the DP-replica line, guarded so that it can never cost the DP
    record: an exception on a rank is agreed through one all_reduce and recorded as {"error": ...};
    a rank that hangs (a collective some rank never reaches) is bounded by a watchdog that prints
    the DP line with {"error": "timeout"} on rank 0 and ends every rank's process."""
    import threading
    limit = float(os.environ.get("GRACE_BENCH_SHARDED_LIMIT", "120"))

    def expire():
        if rank == 0:
            line[key] = {"error": f"timeout: the {key} leg did not finish within {limit:.0f} s"}
            print(json.dumps(line), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)   # non-zero: a hung leg must not read as success (the DP line is printed already)

    dog = threading.Timer(limit, expire)
    dog.daemon = True
    dog.start()
    err = None
    try:
        if os.environ.get("GRACE_BENCH_INJECT_SHARDED_FAILURE", "") in ("all", str(rank)):
            raise RuntimeError(f"injected failure on rank {rank}")
        sh = (fn or bench_topk_sharded)(args, world, rank, dev)
    except Exception as e:          # recorded, not raised: the DP-replica record stays
        err = f"{type(e).__name__}: {e}"[:400]
    flag = torch.tensor([1.0 if err else 0.0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    dog.cancel()
    if float(flag.item()) > 0:
        return {"error": err or "failed on another rank"}
    return {k: sh[k] for k in ("metric", "value", "unit", "ms_per_step", "scaling", "config", "roofline",
                               "shard_decode") if k in sh}


def bench_sharded_codec(args, world, rank, dev, codec):
    """configs[2]'s 161 ResNet-50 tensors as ONE bucket whose elements are split over the
    ranks (grace_amd/dist/sharded_terngrad.py, sharded_quant.py), the decoded bucket replicated on
    every rank; strong scaling (the bucket is fixed).  Bytes per GPU: the shard's encode (TernGrad:
    two reads of x and the codes, 9 B per element; QSGD: 5 B) plus the replicated decode of the
    whole bucket (1 B of codes read, 4 B written per element)."""
    sizes = [int(torch.Size(s).numel()) for s in resnet50_shapes()]
    n = sum(sizes)
    if codec == "terngrad":
        from grace_amd.dist.sharded_terngrad import ShardedTernGrad
        eng = ShardedTernGrad(seed=7)
        enc_b = 9.0
    else:
        from grace_amd.dist.sharded_quant import ShardedQuant
        eng = ShardedQuant("qsgd", quantum_num=127, bucket_size=128, seed=7)
        enc_b = 5.0
    lo, hi = eng.partition(sizes)[rank]
    gen = torch.Generator(device=dev)
    shards = []
    for j in range(args.buffers):
        gen.manual_seed(500 * rank + j + 1)
        shards.append(torch.randn(hi - lo, device=dev, generator=gen) * 0.01)
    elapsed = timed(lambda i: eng.step(shards[i % args.buffers], sizes), args.steps, args.warmup, world, dev)
    t = elapsed / args.steps
    m = max(b - a for a, b in eng.partition(sizes))
    per_gpu = enc_b * m + 5.0 * n
    return {"metric": f"grad-codec GB/s (device-resident encode+decode), {codec} over the ResNet-50 set sharded",
            "value": round(4.0 * n / t / 1e9, 2), "unit": "GB/s", "ms_per_step": round(t * 1e3, 4),
            "scaling": "strong",
            "config": {"workload": f"Sharded{'TernGrad (2-bit packed codes on the wire)' if codec == 'terngrad' else 'Quant(qsgd 127, bucket 128)'}: "
                                   f"161 ResNet-50 tensors ({n} elements) as one bucket over {world} rank(s), "
                                   "replicated dense decode (BASELINE configs[2], SURVEY §8e)",
                       "numel": n, "shard_max": m, "parallelism": f"{world} contiguous unit-aligned shards"},
            "roofline": {"bound": "hbm", "achieved": round(per_gpu / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(per_gpu / t / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_gpu": per_gpu}}


# GRACE_BENCH_NO_PROBE=1: skip the in-bench HBM probes (profiling passes, whose per-dispatch
# counters would otherwise include the probe kernels)
NO_PROBE = os.environ.get("GRACE_BENCH_NO_PROBE", "0") not in ("", "0")


# the round whose PMC passes (tools/r06_session.sh pmc -> profiles/r06_pmc_secondary.json) this
# tree's lines quote: older passes measured older kernels, and some of them another output mode
PMC_TAG = "r06"


def pmc_traffic(workload, alg_bytes, mode=None):
    """HBM bytes per step of a secondary workload's kernels from this round's committed rocprofv3
    FETCH_SIZE / WRITE_SIZE passes (tools/pmc_all.py), with the ratio to the algorithmic bytes.  A
    workload whose step has several output modes (the recycled or dense output of top-k, sharded
    top-k and random-k) passes the mode that ran, and only a pass recorded in that same mode counts:
    a pass of another mode moved other bytes (the no-memory line once quoted an r02
    dense-output pass for the recycled step).  Returns (bytes, ratio, source) or (None, None, None)."""
    path = os.path.join(ROOT, "profiles", f"{PMC_TAG}_pmc_secondary.json")
    try:
        with open(path) as f:
            wl = json.load(f)["workloads"][workload]
    except (OSError, ValueError, KeyError):
        return None, None, None
    if mode is not None and wl.get("mode") != mode:
        return None, None, None
    t = wl["hbm_bytes_per_step"]
    return t, round(t / alg_bytes, 3), os.path.relpath(path, ROOT)


def gpu_clocks(dev):
    """The device's current shader / memory clock levels from sysfs (pp_dpm_sclk / pp_dpm_mclk, the
    level marked '*'), read right after a timed region: VERDICT r4 item 4 (the main pass is bimodal
    across boxes).  Found through the device's PCI address; None where sysfs does not show it."""
    try:
        p = torch.cuda.get_device_properties(dev)
        dom, bus, devid = (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", None),
                           getattr(p, "pci_device_id", None))
        if bus is None or devid is None:
            return None
        base = f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{devid:02x}.0"
        out = {"pci": base.rsplit("/", 1)[1]}
        for clk in ("sclk", "mclk", "fclk", "socclk"):
            try:
                with open(f"{base}/pp_dpm_{clk}") as f:
                    rows = [r.strip() for r in f if r.strip()]
                cur = [r for r in rows if r.endswith("*")]
                out[f"{clk}_current"] = cur[0].split(":", 1)[1].strip(" *") if cur else None
                out[f"{clk}_levels"] = len(rows)
            except OSError:
                out[f"{clk}_current"] = None
        return out
    except Exception as e:   # diagnostics only: never fail the bench line
        return {"error": str(e)[:120]}


def base_line(args, world, elapsed, nbytes_per_rank, metric=METRIC):
    ms = elapsed / args.steps * 1e3
    return {
        "metric": metric, "value": round(world * nbytes_per_rank * args.steps / elapsed / 1e9, 2), "unit": "GB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (torch.randn, buckets rotated per rank)",
    }


# ------------------------------------------------------------------------------------------ top-k
def bench_topk(args, world, rank, dev):
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

    for i in range(args.buffers):       # every name's first step has no residual
        step(i)
    for i in range(args.warmup):        # warm-up steps, untimed and outside the kernel timer
        step(i)
    rec = comm.compressor._recycler
    hits0, dense0 = rec.hits, rec.dense_hits
    ops.timer_enable(True)
    elapsed = timed(step, args.steps, 0, world, dev)
    main_ms, launches = ops.timer_collect()
    ops.timer_enable(False)
    clocks = gpu_clocks(dev)
    # world 1: each step's result is consumed and dropped, so every timed step reuses its bucket's
    # previous result (ops.OutputRecycler): the main pass writes only its selection into the output
    recycled = world == 1 and rec.hits - hits0 == args.steps
    kept = world == 1 and rec.dense_hits - dense0 == args.steps

    line = base_line(args, world, elapsed, 4.0 * n)
    line["config"] = {"workload": "Allgather(TopK 1%, ResidualMemory).step on a 256 MiB fp32 bucket "
                                  "(BASELINE configs[1])",
                      "numel": n, "k": k, "parallelism": f"dp{world} replicas, RCCL allgather of payloads",
                      "output": ("recycled: each step's dropped result is handed back; its k previous non-zeros "
                                 "are cleared and only the new selection is written (bit-identical)")
                      if recycled else ("dense output every step, written in full into the buffer of the bucket's "
                                        "dropped previous result (kept for its placement, ops.pick_pair)"
                                        if kept else "fresh dense output every step")}
    if comm.compressor.place_probes:
        # per bucket: the streaming probe's microseconds for every (residual, output) allocation pair
        # tried at its first step; the fastest pair was kept
        line["config"]["placement_probe_us"] = {nm: [round(x, 1) for x in us]
                                                for nm, us in comm.compressor.place_probes.items()}
    # roofline of the dominant kernel (topk_main), HIP events on the stream it runs on; only the
    # timed steps are counted (warm-up launches ran with the timer off)
    main_avg_ms = main_ms / max(launches, 1)
    # g, r read; r' written; the dense output at world 1 -- all n elements (16 B), or with the
    # recycled output only the selected ones (12 B + 4 B per selected element, ~k)
    if world > 1:
        main_bytes = 12 * n
    elif recycled:
        main_bytes = 12 * n + 4 * k
    else:
        main_bytes = 16 * n
    achieved = main_bytes / (main_avg_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "topk_main", "kernel_avg_us": round(main_avg_ms * 1e3, 2), "launches": launches,
                "algorithmic_bytes_per_launch": main_bytes}
    if world == 1:
        # SURVEY.md §8d config 2 counts 16n + 16k (dense output); recycled: 12n for g, r, r', the
        # payload 8k, the previous payload's indices read 4k and its positions cleared 4k, the new
        # selection written 4k
        step_bytes = 12 * n + 20 * k if recycled else 16 * n + 16 * k
        roofline["step_algorithmic_bytes"] = step_bytes
        roofline["step_frac"] = round(step_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)
        roofline["step_frac_of_16n"] = round((16 * n + 16 * k) / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)
    prof = os.path.join(ROOT, "profiles", "pmc_topk_main.json")
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                pmc = json.load(f)
            if pmc.get("numel") == n and pmc.get("world") == world and pmc.get("recycled", False) == recycled:
                roofline["traffic"] = pmc["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            pass
    # the fraction against a bandwidth measured on this box as well -- the main
    # pass's own streaming skeleton (same kernel, chunking, loads and stores, no classification),
    # each launch right after a real step, timed like the main pass
    skel, skel_med = (skeleton_ceiling(step, main_bytes, n, dev, sparse=recycled) if not NO_PROBE and world == 1
                      else (None, None))
    roofline["measured_copy_gbs"] = skel
    roofline["measured_copy_median_gbs"] = skel_med
    roofline["measured_copy_kind"] = ("grace_topk_stream_probe: the topk_main kernel itself with the classification "
                                      "compiled out (same grid, chunks, 16-B non-temporal loads / stores of g, r, r'"
                                      + (", out untouched as with the recycled output" if recycled else ", out") +
                                      ") on 3 rotated 256 MiB buffer sets (r / out of each placed by ops.pick_pair, "
                                      "as the engine places its own), each launch interleaved with a real "
                                      "step, dispatch-packet events like the main pass; ceiling = fastest launch")
    roofline["frac_of_measured_copy"] = round(achieved / skel, 4) if skel else None
    roofline["frac_of_measured_copy_median"] = round(achieved / skel_med, 4) if skel_med else None
    line["roofline"] = roofline
    line["clocks"] = clocks
    if world == 1 and not args.no_overlap:
        line["two_streams"] = bench_topk_two_streams(args, grads, names)
    line["cpu_baseline"] = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_steps > 0:
        line["cpu_baseline"] = cpu_baseline_topk(n, args.ratio, args.cpu_baseline_steps)
    return line


def bench_topk_two_streams(args, grads, names):
    """The same step sequence with two buckets in flight: bucket j's steps always on
    stream j % 2 (per-stream workspaces, per-name order kept), as a DDP iteration with several
    buckets can issue them.  Reported beside the serial headline, never as `value`; the first
    rotation is checked bit-exact against the serial engine."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory

    dev = grads[0].device
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    comm = Allgather(TopKCompressor(args.ratio), ResidualMemory(), 1)
    ref = Allgather(TopKCompressor(args.ratio), ResidualMemory(), 1)
    torch.cuda.synchronize()

    def step(i):
        j = i % len(grads)
        with torch.cuda.stream(streams[j % 2]):
            return comm.step(grads[j], names[j])

    exact = True
    for i in range(2 * len(grads)):          # first steps (no residual), then with residual
        o = step(i)
        torch.cuda.synchronize()
        exact = exact and torch.equal(o, ref.step(grads[i % len(grads)], names[i % len(grads)]))
    del ref
    elapsed = timed(step, args.steps, args.warmup, 1, dev)
    ms = elapsed / args.steps * 1e3
    return {"ms_per_step": round(ms, 4), "value": round(4.0 * grads[0].numel() / (ms * 1e-3) / 1e9, 2),
            "unit": "GB/s", "streams": 2, "bit_exact_vs_serial": bool(exact),
            "note": "bucket j on stream j % 2; not the headline value (that is one stream, in order)"}


def skeleton_ceiling(step, main_bytes, n, dev, sets=3, rounds=12, sparse=False):
    """The main pass's streaming ceiling on this box: grace_topk_stream_probe (topk_main with the
    classification compiled out: the same grid, loads and stores) on `sets` rotated buffer sets of
    n floats (g, r, out: 768 MiB each, more than the Infinity Cache), each launch right after a real
    step so it runs at the same clocks, timed with the library's dispatch-packet events exactly as
    the main pass is.  Returns (GB/s of the fastest launch, GB/s of the median launch)."""
    from grace_amd import _lib, ops
    bufs = []
    for _ in range(sets):
        g = torch.zeros(n, dtype=torch.float32, device=dev)
        # r and out placed as the engine places its own (ops.pick_pair), so the ceiling is the
        # best-placed layout's, not a chance placement's
        r, o = ops.pick_pair(g)[:2] if ops.PLACE_PROBE and n >= ops.PLACE_MIN_N else (torch.zeros_like(g),
                                                                                        torch.zeros_like(g))
        bufs.append((g, r, o))
    ws = torch.zeros(int(_lib.query("grace_topk_stream_probe_workspace_bytes", n)), dtype=torch.uint8, device=dev)
    ts = []
    for i in range(rounds + sets):
        step(i)
        g, r, o = bufs[i % sets]
        ops.timer_enable(True)
        _lib.call("grace_topk_stream_probe", g.data_ptr(), r.data_ptr(), o.data_ptr(), n, 1 if sparse else 0,
                  ws.data_ptr(), ws.numel(), ops._stream())
        ms, cnt = ops.timer_collect()
        ops.timer_enable(False)
        if i >= sets and cnt == 1:
            ts.append(ms * 1e-3)
    del bufs, ws
    if not ts:
        return None, None
    return round(main_bytes / min(ts) / 1e9, 1), round(main_bytes / sorted(ts)[len(ts) // 2] / 1e9, 1)


def measured_encode_gbs(dev, n, sets=4, reps=7):
    """The box's ceiling for the encoders' traffic mix (QSGD / TernGrad compress: read 4 B, write 1 B
    per element): ``grace_hbm_probe`` variants 6-9 (non-temporal 16-B loads, one byte stored per
    element, no arithmetic) over `sets` rotated buffer sets of `n` floats, the fastest variant's
    median over `reps` launches.  Returns (GB/s counting 5 B per element, variant)."""
    from grace_amd import _lib, ops
    bufs = [(torch.zeros(n, dtype=torch.float32, device=dev), torch.zeros(n // 4 + 16, dtype=torch.float32, device=dev))
            for _ in range(sets)]
    best, best_v = 0.0, None
    for variant in range(6, 10):
        elems = int(_lib.query("grace_hbm_probe_elems", n, variant))
        ts = []
        for i in range(reps + sets):
            g, o = bufs[i % sets]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            _lib.call("grace_hbm_probe", g.data_ptr(), g.data_ptr(), o.data_ptr(), n, variant, ops._stream())
            b.record()
            b.synchronize()
            if i >= sets:
                ts.append(a.elapsed_time(b) * 1e-3)
        gbs = 5.0 * elems / sorted(ts)[len(ts) // 2] / 1e9
        if gbs > best:
            best, best_v = gbs, variant
    del bufs
    return round(best, 1), best_v


def host_cores():
    """(threads to use, how they were chosen): the physical cores of the CPUs this process may run
    on (its affinity mask, SMT siblings counted once), capped by OMP_NUM_THREADS when the box sets
    it (the GPU box grants 16 CPUs of a larger host and exports that share there)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", c))
    phys = max(1, len(cores))
    why = f"{phys} physical cores in this process's affinity mask ({len(cpus)} logical CPUs)"
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < phys:
        why += f", capped at OMP_NUM_THREADS={omp} (the box's CPU share)"
        phys = int(omp)
    return phys, why


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline_topk(n, ratio, steps):
    """The oracle's top-k + residual step on the host cores over the same bucket size."""
    import numpy as np
    from oracle import grace_oracle as O
    threads, why = host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    g = rng.standard_normal(n, dtype=np.float32)
    r = (0.1 * rng.standard_normal(n, dtype=np.float32)).astype(np.float32)
    O.topk_residual_step(g[: 1 << 20], r[: 1 << 20], ratio)     # warm
    t0 = time.perf_counter()
    for _ in range(steps):
        _, _, _, r, _ = O.topk_residual_step(g, r, ratio)
    dt = (time.perf_counter() - t0) / steps
    torch.set_num_threads(prev)
    return {"value": round(4.0 * n / dt / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "cores_chosen": why, "cpu_model": cpu_model(),
            "sample": f"{steps} full 256 MiB top-k 1% + residual steps of oracle/grace_oracle.py "
                      f"(numpy partition + torch CPU ops, {threads} torch threads), {dt * 1e3:.0f} ms/step",
            "note": "conservative: the oracle's numpy partition is faster than the reference's torch.topk "
                    "path (SURVEY.md §6 timed the reference itself at 1,843 ms/step on the 8-core build container)"}


def bench_topk_nomem(args, world, rank, dev):
    """Allgather(TopK 1 %, NoneMemory).step on the 256 MiB bucket ('top-k 1 %
    c+d, no memory'): at world 1 one streaming pass reads g and writes the dense result."""
    from grace_amd import ops
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.none import NoneMemory

    n = args.numel
    k = ops.ratio_k(n, args.ratio)
    comm = Allgather(TopKCompressor(args.ratio), NoneMemory(), world)
    gen = torch.Generator(device=dev)
    grads = []
    for j in range(args.buffers):
        gen.manual_seed(1000 * rank + j + 1)
        grads.append(torch.randn(n, device=dev, generator=gen))

    def step(i):
        return comm.step(grads[i % args.buffers], "bucket")

    def step_unfused(i):            # the reference's four calls (compress, then send_receive)
        payload, ctx = comm.compressor.compress(grads[i % args.buffers], "bucket")
        return comm.send_receive(payload, "bucket", ctx)

    for i in range(args.warmup):
        step(i)
    rec = comm.compressor._recycler
    hits0 = rec.hits
    ops.timer_enable(True)
    elapsed = timed(step, args.steps, 0, world, dev)
    main_ms, launches = ops.timer_collect()
    ops.timer_enable(False)
    recycled = world == 1 and rec.hits - hits0 == args.steps
    # (profiling passes skip the comparison: its kernels would mix into the step's per-kernel counters)
    t_unfused = None if os.environ.get("GRACE_BENCH_NO_UNFUSED") else timed(step_unfused, args.steps, args.warmup, world, dev)
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric="grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket, top-k 1 %, no memory")
    line["config"] = {"workload": "Allgather(TopK 1%, NoneMemory).step on a 256 MiB fp32 bucket (BASELINE.md section 4)",
                      "numel": n, "k": k,
                      "unfused_ms_per_step": round(t_unfused / args.steps * 1e3, 4) if t_unfused else None}
    # 8n + 16k; with the recycled output (each dropped result handed back)
    # the dense write shrinks to the selection: 4n + payload 8k + previous indices 4k + their clear
    # 4k + the new selection 4k
    step_bytes = 4 * n + 20 * k if recycled else 8 * n + 16 * k
    line["config"]["output"] = "recycled" if recycled else "fresh dense output every step"
    main_avg_ms = main_ms / max(launches, 1)
    main_bytes = (4 * n + 4 * k if recycled else 8 * n) if world == 1 else 4 * n
    t = elapsed / args.steps
    traffic, ratio, tsrc = pmc_traffic("topk_nomem", step_bytes, mode="recycled" if recycled else "dense")
    line["roofline"] = {"bound": "hbm", "achieved": round(step_bytes / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(step_bytes / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc,
                        "step_algorithmic_bytes": step_bytes, "kernel": "topk_main",
                        "kernel_avg_us": round(main_avg_ms * 1e3, 2),
                        "kernel_frac": round(main_bytes / (main_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        # BASELINE.md section 4's definition of this row (>= 70 % target): 8n + 16k
                        # per step whatever the output mode
                        "baseline_bytes": 8 * n + 16 * k,
                        "frac_of_baseline_bytes": round((8 * n + 16 * k) / t / 1e9 / HBM_PEAK_GBS, 4)}
    return line


def bench_topk_e2e(args, world, rank, dev):
    """H2D (pinned) -> Allgather(TopK, Residual).step -> D2H (pinned), serial on the current stream."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    n = args.numel
    comm = Allgather(TopKCompressor(args.ratio), ResidualMemory(), world)
    hosts = [torch.randn(n).pin_memory() for _ in range(2)]
    back = torch.empty(n).pin_memory()
    dbuf = torch.empty(n, device=dev)

    def step(i):
        dbuf.copy_(hosts[i % 2], non_blocking=True)
        out = comm.step(dbuf, "bucket")
        back.copy_(out, non_blocking=True)

    step(0)
    elapsed = timed(step, args.steps, args.warmup, world, dev)
    # the copies alone, for the split
    def copies(i):
        dbuf.copy_(hosts[i % 2], non_blocking=True)
        back.copy_(dbuf, non_blocking=True)
    t_copy = timed(copies, args.steps, args.warmup, world, dev)
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric="grad-codec GB/s (host-resident bucket: H2D + encode+decode + D2H), 256 MiB fp32")
    line["config"] = {"workload": "pinned host bucket -> H2D -> Allgather(TopK 1%, ResidualMemory).step -> D2H",
                      "numel": n, "h2d_plus_d2h_ms": round(t_copy / args.steps * 1e3, 4)}
    line["roofline"] = None
    line["pipelined"] = bench_topk_e2e_pipelined(args, world, dev)
    return line


def bench_topk_e2e_pipelined(args, world, dev):
    """The same per-bucket work as a DDP loop sees it: bucket i's H2D on a copy-in stream, its step on
    the compute stream, its D2H on a copy-out stream, so bucket i + 1 arrives while bucket i computes
    and bucket i - 1 leaves (PCIe is full duplex).  Three buckets with their own residuals rotate;
    events order each bucket's three stages and the reuse of its device buffer."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    n = args.numel
    comm = Allgather(TopKCompressor(args.ratio), ResidualMemory(), world)
    nb = 3
    hosts = [torch.randn(n).pin_memory() for _ in range(nb)]
    backs = [torch.empty(n).pin_memory() for _ in range(nb)]
    dbufs = [torch.empty(n, device=dev) for _ in range(nb)]
    s_in, s_cmp, s_out = (torch.cuda.Stream(device=dev) for _ in range(3))
    done = [None] * nb          # event: bucket b's step has finished reading dbufs[b]
    left = [None] * nb          # event: bucket b's last D2H out of backs[b] has finished

    def step(i):
        b = i % nb
        with torch.cuda.stream(s_in):
            if done[b] is not None:
                s_in.wait_event(done[b])
            dbufs[b].copy_(hosts[b], non_blocking=True)
            arrived = torch.cuda.Event()
            arrived.record(s_in)
        with torch.cuda.stream(s_cmp):
            s_cmp.wait_event(arrived)
            out = comm.step(dbufs[b], f"bucket{b}")
            computed = torch.cuda.Event()
            computed.record(s_cmp)
            done[b] = computed
        with torch.cuda.stream(s_out):
            s_out.wait_event(computed)
            if left[b] is not None:
                s_out.wait_event(left[b])
            backs[b].copy_(out, non_blocking=True)
            out.record_stream(s_out)
            ev = torch.cuda.Event()
            ev.record(s_out)
            left[b] = ev

    for i in range(nb):
        step(i)
    torch.cuda.synchronize(dev)
    elapsed = timed(step, args.steps, args.warmup, world, dev)
    t = elapsed / args.steps
    return {"ms_per_step": round(t * 1e3, 4), "value": round(4.0 * n / t / 1e9, 2), "unit": "GB/s",
            "streams": 3, "buckets": nb,
            "note": "H2D of bucket i+1, the step of bucket i and the D2H of bucket i-1 overlap (copy-in, compute, "
                    "copy-out streams); the serial line above runs the three one after the other"}


def bench_topk_sharded(args, world, rank, dev):
    from grace_amd.dist.sharded import ShardedTopK
    n = args.numel
    ratio = 0.001 if args.ratio == 0.01 else args.ratio
    sizes = [n // world + (1 if r < n % world else 0) for r in range(world)]
    m = sizes[rank]
    eng = ShardedTopK(ratio)
    gen = torch.Generator(device=dev)
    shards = []
    for j in range(args.buffers):
        gen.manual_seed(1000 * rank + j + 1)
        shards.append(torch.randn(m, device=dev, generator=gen))
    for j in range(args.buffers):
        eng.step(shards[j], f"b{j}")
    elapsed = timed(lambda i: eng.step(shards[i % args.buffers], f"b{i % args.buffers}"), args.steps, args.warmup,
                    world, dev)
    t = elapsed / args.steps
    k = max(1, int(n * ratio))
    line = base_line(args, 1, elapsed, 4.0 * n,
                     metric="grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket sharded, top-k 0.1 %")
    line["n_gpus"] = world
    line["scaling"] = "strong"
    line["config"] = {"workload": f"ShardedTopK(0.1 %) + residual, one {4 * n >> 20} MiB bucket over {world} "
                                  "rank(s), replicated dense decode (BASELINE configs[4])",
                      "numel": n, "k": k, "shard": m, "parallelism": f"{world} contiguous shards"}
    survey = 12.0 * m + 8.0 * k + 4.0 * n       # shard encode + replicated decode
    recycled = eng._recycler.hits > 0
    if recycled:
        # the dropped output comes back (ShardedTopK.recycle_output): instead of a 4n zero-fill, the
        # select reads the W records (8 B per entry), writes every entry's selection record (4 B) and
        # the next step's clear reads it (4 B); k new values in, k old ones out (4 B each)
        per_gpu = 12.0 * m + 8.0 * k + 16.0 * world * k + 8.0 * k
    else:
        per_gpu = survey
    traffic, t_ratio, tsrc = (pmc_traffic("topk_sharded", per_gpu, mode="recycled" if recycled else "dense")
                              if world == 1 else (None, None, None))
    line["roofline"] = {"bound": "hbm", "achieved": round(per_gpu / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(per_gpu / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": t_ratio, "traffic_source": tsrc,
                        "algorithmic_bytes_per_gpu": per_gpu, "survey_bytes_per_gpu": survey,
                        "output": "recycled" if recycled else "dense zero-fill",
                        "recycled_steps": eng._recycler.hits}
    # SURVEY §8e's sharded-decode mode beside it: every rank materialises only its own n/W slice of
    # the decoded bucket (reduce-scatter semantics), same selection, same single collective
    eng_s = ShardedTopK(ratio, dense="shard")
    for j in range(args.buffers):
        eng_s.step(shards[j], f"s{j}")
    el_s = timed(lambda i: eng_s.step(shards[i % args.buffers], f"s{i % args.buffers}"), args.steps, args.warmup,
                 world, dev)
    t_s = el_s / args.steps
    per_gpu_s = 12.0 * m + 8.0 * k + 4.0 * m          # shard encode + the own slice of the decode
    line["shard_decode"] = {"value": round(4.0 * n / t_s / 1e9, 2), "unit": "GB/s", "ms_per_step": round(t_s * 1e3, 4),
                            "frac": round(per_gpu_s / t_s / 1e9 / HBM_PEAK_GBS, 4),
                            "algorithmic_bytes_per_gpu": per_gpu_s,
                            "note": "ShardedTopK(dense='shard'): each rank decodes only its own slice"}
    return line


def bench_ddp(args, world, rank, dev):
    from grace_amd.dist.helper import grace_from_params
    from grace_amd.dist.segmented import SegmentedTopK
    from grace_amd.harness import GradBucket, ShapeModel, step_bucketed, step_parameters, step_segmented
    model = ShapeModel(resnet50_shapes(), dev)
    bucket = GradBucket(model)
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                             "communicator": "allgather", "world_size": world})
    bucket.flat.normal_()
    if args.workload == "ddp_params":
        fn = lambda i: step_parameters(model, grc)   # noqa: E731
    elif args.workload == "ddp_segmented":
        eng = SegmentedTopK(0.01, world_size=world)
        fn = lambda i: step_segmented(bucket, eng)   # noqa: E731
    else:
        fn = lambda i: step_bucketed(bucket, grc)    # noqa: E731
    fn(0)
    elapsed = timed(fn, args.steps, args.warmup, world, dev)
    total = bucket.flat.numel()
    line = base_line(args, world, elapsed, 4.0 * total,
                     metric=f"grad-codec GB/s, ResNet-50 gradients through the DDP loopback harness ({args.workload})")
    kind = {"ddp_params": "per-parameter grc.step loop (core.py:204-208)",
            "ddp_segmented": "per-tensor k and residual, all tensors in one launch sequence (SegmentedTopK)",
            "ddp_bucket": "one flat bucket, ONE global top-k (a different algorithm)"}[args.workload]
    line["config"] = {"workload": f"{kind}, Allgather(TopK 1 %, Residual), 161 ResNet-50 tensors", "numel": total,
                      "tensors": len(bucket.params)}
    # algorithmic bytes: read g, r; write r' and (world 1) the dense output; the payload (8 B per
    # selected entry: per-tensor k_i, or one global k for ddp_bucket)
    if args.workload == "ddp_bucket":
        k_sum = max(1, int(total * 0.01))
    else:
        k_sum = sum(min(p.numel(), max(1, int(p.numel() * 0.01))) for p in bucket.params)
    alg = (16 if world == 1 else 12) * total + 8 * k_sum
    t = elapsed / args.steps
    traffic, ratio, tsrc = pmc_traffic(args.workload, alg) if world == 1 else (None, None, None)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc,
                        "algorithmic_bytes_per_step": alg, "selected_per_step": k_sum,
                        "note": "16 B per element at world 1 (g, r read; r', dense out written) + 8 B per selected entry"}
    return line


# ------------------------------------------------------------------------------------------ sign
def bench_sign(args, world, rank, dev):
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    n = (1 << 20) if args.workload == "sign" else args.numel
    comm = Allgather(SignSGDCompressor(), NoneMemory(), world)
    nbuf = max(args.buffers, 64 if n <= (1 << 20) else 3)     # 4 MiB buckets: rotate past the MALL
    grads = [torch.randn(n, device=dev) for _ in range(nbuf)]
    if n <= (1 << 20):
        # launch-bound (~5 us per step): a short untimed pre-warm so a 20-step timing sees the
        # steady launch path and clocks rather than the first few hundred microseconds of them
        for i in range(200):
            comm.step(grads[i % nbuf], "w")
    elapsed = timed(lambda i: comm.step(grads[i % nbuf], "w"), args.steps, args.warmup, world, dev)
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric=f"grad-codec GB/s (device-resident encode+decode), {4 * n >> 20} MiB fp32 signSGD")
    line["config"] = {"workload": f"Allgather(SignSGD, NoneMemory).step, {4 * n >> 20} MiB fp32", "numel": n,
                      "rotated_buffers": nbuf}
    t = elapsed / args.steps
    # the world-1 fused step never materialises the u8 codes: it reads x and writes the result, 8n.
    # `frac` follows the bytes moved; SURVEY.md §8d's 10n (the codes written and read back) is kept
    # beside it as frac_of_survey_bytes (a frac on 10n printed an `achieved` above the
    # box's measured copy rate)
    alg = 8.0 * n if world == 1 else 10.0 * n
    traffic, ratio, tsrc = pmc_traffic(args.workload, alg)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_over_algorithmic": ratio, "traffic_source": tsrc,
                        "algorithmic_bytes_per_step": alg,
                        "frac_of_survey_bytes": round(10.0 * n / t / 1e9 / HBM_PEAK_GBS, 4),
                        "note": ("8n moved per step at world 1 (x read, the f32 result written; the fused step "
                                 "never stores the u8 codes); frac_of_survey_bytes counts SURVEY.md §8d config 1's "
                                 "10n" if world == 1 else "10n: the u8 codes written and read back")}
    return line


# ------------------------------------------------------------------------------------------ QSGD / TernGrad
def bench_quant(args, world, rank, dev):
    from grace_amd import ops
    shapes = resnet50_shapes()
    sizes = [int(torch.Size(s).numel()) for s in shapes]
    total = sum(sizes)
    nbuf = 3
    flats = [torch.randn(total, device=dev) * 0.01 for _ in range(nbuf)]
    if args.workload == "qsgd_step":
        # world-1 Allgather(QSGD(127, 128)).step fused (grace_qsgd_step_w1): x read once, out written once
        def step(i):
            return ops.qsgd_step_w1(flats[i % nbuf], 127, sizes=sizes, seed=i)
        alg = 8 * total
    elif args.workload == "terngrad_step":
        # statistics pass (read x) + fused encode/decode pass (read x, write out)
        def step(i):
            return ops.terngrad_step_w1(flats[i % nbuf], sizes=sizes, seed=i)
        alg = 12 * total + 4 * len(sizes)
    elif args.workload == "qsgd":
        def step(i):
            x = flats[i % nbuf]
            codes, norms = ops.qsgd_compress(x, 127, 128, sizes=sizes, seed=i)
            return ops.qsgd_decompress(codes, norms, 127, 128, total, sizes=sizes)
        nb = sum((s + 127) // 128 for s in sizes)
        alg = 10 * total + 8 * nb
    else:
        def step(i):
            x = flats[i % nbuf]
            codes, scal = ops.terngrad_compress(x, sizes=sizes, seed=i)
            return ops.terngrad_decompress(codes, scal, total, sizes=sizes)
        alg = 10 * total + 8 * len(sizes)
    elapsed = timed(step, args.steps, args.warmup, world, dev)
    t = elapsed / args.steps
    line = base_line(args, world, elapsed, 4.0 * total,
                     metric=f"grad-codec GB/s (device-resident encode+decode), ResNet-50 set {args.workload}")
    what = ("world-1 fused Allgather step (codes never stored)" if args.workload.endswith("_step")
            else "compress+decompress")
    line["config"] = {"workload": f"{args.workload} {what}, 161 ResNet-50 tensors in one segmented "
                                  "launch per stage (BASELINE configs[2])", "numel": total, "tensors": len(sizes)}
    traffic, ratio, tsrc = pmc_traffic(args.workload, alg)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc, "algorithmic_bytes_per_step": alg}
    # the encoders' own ceiling: the same read-4-B / write-1-B mix streamed with no arithmetic
    if not NO_PROBE:
        enc_gbs, enc_v = measured_encode_gbs(dev, total)
        line["roofline"].update({"measured_encode_mix_gbs": enc_gbs, "measured_encode_mix_variant": enc_v,
                                 "encode_floor_us": round(5.0 * total / enc_gbs / 1e3, 2)})
    return line


# ------------------------------------------------------------------------------------------ natural / cnat / fp16
def bench_cast(args, world, rank, dev):
    """Allgather(NaturalCompressor | NaturalCompressor_CUDA | FP16Compressor, NoneMemory).step on a 256 MiB
    bucket: element-wise codecs, u8 codes (natural, cnat) or f16 (fp16)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.fp16 import FP16Compressor
    from grace_amd.dist.compressor.natural import NaturalCompressor, NaturalCompressor_CUDA
    from grace_amd.dist.memory.none import NoneMemory
    n = args.numel
    comp = {"natural": NaturalCompressor, "cnat": NaturalCompressor_CUDA, "fp16": FP16Compressor}[args.workload]()
    comm = Allgather(comp, NoneMemory(), world)
    nbuf = 3
    grads = [torch.randn(n, device=dev) for _ in range(nbuf)]
    elapsed = timed(lambda i: comm.step(grads[i % nbuf], "w"), args.steps, args.warmup, world, dev)
    t = elapsed / args.steps
    code_bytes = 2 if args.workload == "fp16" else 1
    # world 1 runs the fused step (grace_cast_step_w1: read x, write the decoded f32, the codes never
    # stored) = 8n; otherwise encode + decode move the codes too
    alg = 8 * n if world == 1 else (8 + 2 * code_bytes) * n
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric=f"grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 {args.workload}")
    line["config"] = {"workload": f"Allgather({type(comp).__name__}, NoneMemory).step, 256 MiB fp32", "numel": n,
                      "rotated_buffers": nbuf}
    traffic, ratio, tsrc = pmc_traffic(args.workload, alg)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc, "algorithmic_bytes_per_step": alg,
                        "note": "8n at world 1 (fused step: x read once, the f32 result written once); "
                                f"{8 + 2 * code_bytes}n with the codes materialised (world > 1)"}
    return line


# ------------------------------------------------------------------------------------------ PowerSGD
def ops_ratio_k(n, ratio):
    from grace_amd import ops
    return ops.ratio_k(n, ratio)


def bench_sparse(args, world, rank, dev):
    """SURVEY.md 8a rows a6 / a7 on the 256 MiB bucket with ResidualMemory: Allgather(RandomK 1 %)
    and Allgather(Threshold), the threshold at 2.5758 (|x| above it: 1 % of N(0, 1) on the first
    step; the residual grows it afterwards, as in training)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.memory.residual import ResidualMemory
    n = args.numel
    if args.workload == "randomk":
        from grace_amd.dist.compressor.randomk import RandomKCompressor
        comp = RandomKCompressor(args.ratio)
        desc = "Allgather(RandomK 1%, ResidualMemory).step"
    else:
        from grace_amd.dist.compressor.threshold import ThresholdCompressor
        comp = ThresholdCompressor(2.5758)
        desc = "Allgather(Threshold 2.5758, ResidualMemory).step"
    comm = Allgather(comp, ResidualMemory(), world)
    grads = [torch.randn(n, device=dev) for _ in range(args.buffers)]
    for j in range(args.buffers):
        comm.step(grads[j], f"b{j}")
    elapsed = timed(lambda i: comm.step(grads[i % args.buffers], f"b{i % args.buffers}"), args.steps, args.warmup,
                    world, dev)
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric=f"grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket, {args.workload}")
    line["config"] = {"workload": f"{desc} on a 256 MiB fp32 bucket (SURVEY.md 8a)", "numel": n}
    alg = 16.0 * n                       # g, r read; r', dense out written (payload bytes excluded)
    t = elapsed / args.steps
    rec = getattr(comp, "_recycler", None)
    mode = None
    if args.workload == "randomk":       # random-k's world-1 step recycles its dropped output
        mode = "recycled" if rec is not None and rec.hits > 0 else "dense"
        line["config"]["output"] = mode
        if mode == "recycled":
            # g, r read, r' written (12n); the output: the previous k positions cleared and the new
            # k written (4 B each), the drawn indices written and read back (8 B each with grouping)
            k = ops_ratio_k(n, args.ratio)
            alg = 12.0 * n + 16.0 * k
    if args.workload == "threshold" and getattr(comp, "place_probes", None):
        line["config"]["output"] = ("dense every step, written in full into the bucket's kept buffer (residual / "
                                    "output allocation pair placed by ops.pick_pair)")
        line["config"]["placement_probe_us"] = {nm: [round(x, 1) for x in us] for nm, us in comp.place_probes.items()}
    traffic, ratio, tsrc = pmc_traffic(args.workload, alg, mode=mode)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc, "algorithmic_bytes_per_step": alg,
                        "frac_of_16n": round(16.0 * n / t / 1e9 / HBM_PEAK_GBS, 4)}
    return line


def bench_dgc(args, world, rank, dev):
    """Allgather(DgcCompressor(1 %), DgcMemory(0.9)).step on the 256 MiB
    bucket (grace_dl/dist/compressor/dgc.py:12-50, memory/dgc.py:15-39).  The payload size is data
    dependent (variable-size Allgather, one host read of the count per step, as the reference)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.dgc import DgcCompressor
    from grace_amd.dist.memory.dgc import DgcMemory
    n = args.numel
    comm = Allgather(DgcCompressor(args.ratio), DgcMemory(0.9, False, world), world)
    grads = [torch.randn(n, device=dev) for _ in range(args.buffers)]
    for j in range(args.buffers):
        comm.step(grads[j], f"b{j}")
    elapsed = timed(lambda i: comm.step(grads[i % args.buffers], f"b{i % args.buffers}"), args.steps, args.warmup,
                    world, dev)
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric="grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 bucket, DGC 1 %")
    line["config"] = {"workload": "Allgather(DgcCompressor(1%), DgcMemory(0.9)).step, 256 MiB fp32 (SURVEY.md 8f.3)",
                      "numel": n}
    if world == 1:
        # the world-1 step reads g, r, a and writes r', a', out once (grace_dgc_step_w1_fused): 24 B
        alg = 24.0 * n
        note = ("24n: one pass reads g, r, a and writes r', a' and the dense output (the sampled threshold "
                "stands; otherwise a gated fix-up redoes the step); sample and its top-k excluded")
    else:
        # compensate 20 B (g, r, a read; r, a written), threshold histogram over a 4 B, compaction 4 B,
        # mask update 16 B (r, a), dense decode 4 B
        alg = 48.0 * n
        note = ("48n: compensate 20n, threshold histogram 4n, compaction 4n, mask update 16n, dense decode 4n "
                "(the reference's passes, each fused to one kernel)")
    t = elapsed / args.steps
    traffic, ratio, tsrc = pmc_traffic("dgc", alg)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc, "algorithmic_bytes_per_step": alg, "note": note}
    return line


def bench_sign_bits(args, world, rank, dev):
    """signSGD with the 1-bit wire layout (SignSGDCompressor(wire="bits")),
    compress + Allgather decode on the 256 MiB bucket at world size 1 (the packed payload is what a
    world > 1 exchange would move: n / 8 bytes per rank)."""
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.signsgd import SignSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    n = args.numel
    comm = Allgather(SignSGDCompressor(wire="bits"), NoneMemory(), world)
    grads = [torch.randn(n, device=dev) for _ in range(args.buffers)]

    def step(i):   # the four calls, so the packed payload is produced and decoded
        g = grads[i % args.buffers]
        payload, ctx = comm.compressor.compress(g, "w")
        return comm.send_receive(payload, "w", ctx)

    elapsed = timed(step, args.steps, args.warmup, world, dev)
    line = base_line(args, world, elapsed, 4.0 * n,
                     metric="grad-codec GB/s (device-resident encode+decode), 256 MiB fp32 signSGD, 1-bit wire")
    line["config"] = {"workload": "SignSGD wire='bits': compress (1 bit / element) + Allgather decode, 256 MiB fp32",
                      "numel": n}
    alg = 4.0 * n + n / 8 + n / 8 * world + 4.0 * n     # read x, write bits; read W bit payloads, write out
    t = elapsed / args.steps
    traffic, ratio, tsrc = pmc_traffic("sign_bits", alg)
    line["roofline"] = {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc, "algorithmic_bytes_per_step": alg}
    return line


def bench_powersgd(args, world, rank, dev):
    from grace_amd.dist.communicator.allreduce import Allreduce
    from grace_amd.dist.compressor.powersgd import PowerSGDCompressor
    from grace_amd.dist.memory.none import NoneMemory
    n = m = 4096
    r = 4
    comm = Allreduce(PowerSGDCompressor(rank=r, world_size=world), NoneMemory(), world)
    nbuf = 5   # 5 x 64 MiB rotated: more than the 256 MB MALL holds, so no step reuses the last one's M
    grads = [torch.randn(n, m, device=dev) for _ in range(nbuf)]
    elapsed = timed(lambda i: comm.step(grads[i % nbuf], "w"), args.steps, args.warmup, world, dev)
    t = elapsed / args.steps
    flops = 3 * 2 * n * m * r
    line = base_line(args, world, elapsed, 4.0 * n * m,
                     metric="grad-codec GB/s (device-resident encode+decode), PowerSGD rank 4, 4096x4096")
    line["config"] = {"workload": "Allreduce(PowerSGD rank 4, NoneMemory).step, 4096x4096 fp32 (BASELINE configs[3])",
                      "numel": n * m, "rank": r}
    # the world-1 one-pass compress reads M once (P and the f64 Qraw partials from the same registers)
    # and the decode writes P Q^T: 8 B per element, plus the partials written and read back (64-row
    # slabs x m x r x 8 B); SURVEY.md §8d's 12n (M read twice) is kept as frac_of_survey_bytes
    moved = 8.0 * n * m + 2.0 * (n // 64) * m * r * 8 if world == 1 else 12.0 * n * m
    traffic, ratio, tsrc = pmc_traffic("powersgd", moved)
    line["roofline"] = {"bound": "hbm", "achieved": round(moved / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(moved / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": ratio, "traffic_source": tsrc, "algorithmic_bytes_per_step": moved,
                        "frac_of_survey_bytes": round(12 * n * m / t / 1e9 / HBM_PEAK_GBS, 4),
                        "mfma_tflops": round(flops / t / 1e12, 3),
                        "mfma_util": round(flops / t / 1e12 / F32_PEAK_TFLOPS, 5),
                        "note": "frac on the bytes the one-pass step moves (8 B per element + the f64 partials); "
                                "frac_of_survey_bytes on SURVEY.md §8d config 4's 12n; 6nmr flops (AI = 2 flop/B)"}
    return line


if __name__ == "__main__":
    main()
