"""Per-stage timing of PowerSGD (4096 x 4096, rank 4) for one or more library builds.
usage: python tools/exp_psgd.py [lib.so ...]   (each lib timed in its own subprocess)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import torch
    sys.path.insert(0, ROOT)
    from grace_amd import ops

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e3

    Ms = [torch.randn(4096, 4096, device="cuda") for _ in range(3)]
    q = torch.randn(4096, 4, device="cuda")
    P = ops.powersgd_p(Ms[0], q)
    Q = ops.powersgd_qt(Ms[0], P)
    it = iter(range(10 ** 9))
    A64 = torch.randn(64, 4, device="cuda")
    A16k = torch.randn(16384, 4, device="cuda")
    E = torch.empty(64, device="cuda")
    res = {
        "p": timeit(lambda: ops.powersgd_p(Ms[next(it) % 3], q)),
        "qt": timeit(lambda: ops.powersgd_qt(Ms[next(it) % 3], P)),
        "orth": timeit(lambda: ops.orthogonalize_(P)),
        "outer": timeit(lambda: ops.powersgd_outer(P, Q)),
        "qdraw": timeit(lambda: ops.normal_orthogonal((4096, 4), 5, "cuda")),
        "copy": timeit(lambda: Ms[1].copy_(Ms[next(it) % 2 * 2])),
        "orth64": timeit(lambda: ops.orthogonalize_(A64)),
        "orth16k": timeit(lambda: ops.orthogonalize_(A16k)),
        "empty": timeit(lambda: ops.fill(E, 0.0)),
    }
    print(os.environ.get("GRACE_HIP_LIB", "default"), " ".join(f"{k}={v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
    else:
        libs = sys.argv[1:] or [""]
        for lib in libs:
            env = dict(os.environ)
            if lib:
                env["GRACE_HIP_LIB"] = lib
            subprocess.run([sys.executable, __file__, "--child"], env=env, check=True, timeout=300)
