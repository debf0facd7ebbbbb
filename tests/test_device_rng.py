"""CPU checks of the numpy restatement of the device generator (tests/device_rng.py)."""
import numpy as np

from tests.device_rng import mix64, qsgd_bucket128_uniforms, quad_uniforms


def test_mix64_is_splitmix64():
    # splitmix64's first output from state 0 (the published known answer)
    assert mix64(0) == 0xE220A8397B1DCDAF


def test_quad_uniforms_range_and_quads():
    u = quad_uniforms(7, np.repeat(np.arange(0, 4096, 4), 4), np.tile(np.arange(4), 1024))
    assert u.dtype == np.float32 and u.min() >= 0.0 and u.max() < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.02
    # segments restart the bucket grid: an unaligned segment's quads start at its own bucket base
    v = qsgd_bucket128_uniforms(7, [5, 130])
    assert np.array_equal(v[5:9], quad_uniforms(7, [5] * 4, np.arange(4)))
    assert np.array_equal(v[133:135], quad_uniforms(7, [133] * 2, np.arange(2)))
