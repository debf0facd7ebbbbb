"""Build libgrace_hip.so (all HIP sources under grace_amd/csrc) for gfx950, in-tree.

Plain hipcc, no torch extension machinery: the library has a C ABI (include/grace_hip.h) and is
loaded with ctypes.  Objects are rebuilt only when a source or header is newer.
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libgrace_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
    "-ffp-contract=off",                          # every f32 op rounds like the reference's torch ops
    "-fhip-fp32-correctly-rounded-divide-sqrt",   # IEEE division / sqrt (QSGD, TernGrad scales)
    "-Wall", "-Wno-unused-function",
]


def _newest_dep():
    deps = glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "grace_hip.h")]
    return max(os.path.getmtime(d) for d in deps)


def _compile(src, obj, verbose):
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=False, jobs=8, variant=""):
    """variant "stamps" builds the diagnostic libgrace_hip_stamps.so (-DGRACE_STAMPS)."""
    global FLAGS, LIB
    if variant:
        defs = {"stamps": ["-DGRACE_STAMPS"]}
        extra = os.environ.get("GRACE_BUILD_DEFS", "")
        FLAGS = FLAGS + defs.get(variant, [f"-DGRACE_{variant.upper()}"] if not extra else []) + \
            [f"-D{d}" for d in extra.split(",") if d]
        LIB = os.path.join(LIBDIR, f"libgrace_hip_{variant}.so")
    objdir = os.path.join(LIBDIR, "obj" + (f"_{variant}" if variant else ""))
    os.makedirs(objdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    dep_t = _newest_dep()
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), dep_t):
            todo.append((s, o))
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo) or 1))) as ex:
        list(ex.map(lambda so: _compile(so[0], so[1], verbose), todo))
    if todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    var = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--variant=")), "")
    print(build(verbose="-v" in sys.argv, variant=var))
