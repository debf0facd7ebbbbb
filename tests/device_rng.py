"""numpy restatement of grace_amd's own device generator (grace_amd/csrc/common.h: mix64, fmix32,
rand32, uniform01x4) -- test infrastructure, not the reference's algorithm (the reference draws from
torch's generators; rng="torch_cpu" reproduces those).  It lets the device-generator fast paths be
checked bit for bit: the uniforms a kernel draws on its own equal the ones restated here, so
``compress(x, seed=s)`` must equal ``compress(x, u=quad_uniforms(...))`` exactly."""
import numpy as np

M64 = (1 << 64) - 1


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _fmix32(h):
    h = h.astype(np.uint64)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def _to_u01(h):
    return ((h >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def quad_uniforms(seed, quad_start, lane):
    """uniform01x4(seed, quad_start)[lane] for element indices below 2^32 (rand32's high-word term
    is zero there)."""
    k = mix64(int(seed) & M64)
    klo, khi = np.uint64(k & 0xFFFFFFFF), np.uint64(k >> 32)
    e = np.asarray(quad_start, dtype=np.uint64)
    h = _fmix32((((e * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)) ^ klo) + khi & np.uint64(0xFFFFFFFF))
    lane = np.asarray(lane)
    out = _to_u01(h)
    h = np.where(h == 0, np.uint64(0x9E3779B9), h)
    for j in range(1, 4):
        h ^= (h << np.uint64(13)) & np.uint64(0xFFFFFFFF)
        h ^= h >> np.uint64(17)
        h ^= (h << np.uint64(5)) & np.uint64(0xFFFFFFFF)
        out = np.where(lane == j, _to_u01(h), out)
    return out


def qsgd_bucket128_uniforms(seed, sizes):
    """The uniform each element of the segmented QSGD(bucket 128) encoders draws: the quad of element
    i starts at its bucket's base + 4 * ((i - base) // 4) (grace_amd/csrc/quant.hip)."""
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    seg = np.repeat(np.arange(len(sizes)), sizes)
    i = np.arange(int(np.sum(sizes)), dtype=np.int64)
    rel = i - starts[seg]
    base = starts[seg] + (rel // 128) * 128
    qs = base + ((i - base) // 4) * 4
    return quad_uniforms(seed, qs, i - qs)
