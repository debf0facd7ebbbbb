"""Pin the CPU oracle against golden vectors captured from the reference (CPU-only)."""
import numpy as np
import pytest

from oracle import grace_oracle as O
from tests.golden_util import same_bits, topk_sets_match


# ----------------------------------------------------------------------------- sign family
def test_signsgd_golden(golden):
    cases = golden.cases("sign", codec="signsgd")
    assert len(cases) >= 8
    for c in cases:
        if "codes" not in c:
            continue
        codes = O.sign_encode(c["x"])
        assert np.array_equal(codes, c["codes"].ravel()), c.name
        assert same_bits(O.sign_decode(codes), c["dec"].ravel()), c.name
        decs = [O.sign_decode(O.sign_encode(c[f"agg_in{i}"])) for i in range(3)]
        assert same_bits(O.sign_aggregate(decs), c["agg"].ravel()), c.name


def test_signsgd_step_world1(golden):
    c = golden.case("sign", "signsgd_step_w1")
    out = O.sign_aggregate([O.sign_decode(O.sign_encode(c["x"]))])
    assert same_bits(out, c["out"].ravel())


def test_signum_golden(golden):
    c = golden.case("sign", "signum_seq")
    prev = None
    for s in range(3):
        m = O.signum_momentum(c[f"x{s}"], prev, 0.9)
        assert same_bits(m, c[f"mom{s}"].ravel())
        assert np.array_equal(O.sign_encode(m), c[f"codes{s}"])
        prev = m


def test_efsignsgd_golden(golden):
    c = golden.case("sign", "efsignsgd_seq")
    res = None
    decs = []
    for s in range(3):
        t = O.efsign_compensate(c[f"x{s}"], res, 0.1)
        assert same_bits(t, c[f"t{s}"]), s
        mean, codes = O.efsign_compress(t)
        assert same_bits(mean, c[f"mean{s}"]), s
        assert np.array_equal(codes, c[f"codes{s}"])
        dec = O.efsign_decode(mean, codes)
        assert same_bits(dec, c[f"dec{s}"]), s
        res = O.residual_update(t, dec)
        assert same_bits(res, c[f"res{s}"]), s
        decs.append(dec)
    agg = (O.python_sum(decs) / np.float32(0.1)).astype(np.float32)
    assert np.allclose(agg, c["agg"], rtol=1e-6)


def test_onebit_golden(golden):
    for c in golden.cases("sign", codec="onebit"):
        mask0, m0, m1 = O.onebit_compress(c["x"])
        assert np.array_equal(mask0, c["mask0"]), c.name
        assert same_bits(np.array([m0]), c["mean0"]), c.name
        assert same_bits(np.array([m1]), c["mean1"]), c.name
        assert same_bits(O.onebit_decode(mask0, m0, m1, quirk=True), c["dec_quirk"]), c.name
        assert same_bits(O.onebit_decode(mask0, m0, m1), c["dec_fixed"]), c.name


# ----------------------------------------------------------------------------- sparse
def test_topk_golden(golden):
    cases = golden.cases("sparse", codec="topk", prefix="topk_")
    single = [c for c in cases if "steps" not in c.meta]
    assert len(single) >= 30
    for c in single:
        x = c["x"].ravel()
        k = O.ratio_k(x.size, c.meta["ratio"])
        vals, idx = O.topk_select(x, k)
        assert topk_sets_match(x, idx, c["idx"], k), c.name
        # values are x[idx] bit-exactly
        assert same_bits(vals, x[idx])
        assert same_bits(c["vals"], x[c["idx"].astype(np.int64)])
        # decompressed tensor bit-exact outside of ties; identical where the sets agree
        dec = O.sparse_decode(vals, idx, x.size)
        if np.array_equal(np.sort(idx), np.sort(c["idx"])):
            assert same_bits(dec, c["dec"].ravel()), c.name


def test_topk_residual_sequence(golden):
    for c in golden.cases("sparse", codec="topk"):
        if "steps" not in c.meta:
            continue
        res = None
        for s in range(c.meta["steps"]):
            t, vals, idx, res_new, out = O.topk_residual_step(c[f"g{s}"], res, c.meta["ratio"])
            assert same_bits(t, c[f"t{s}"].ravel()), (c.name, s)
            k = O.ratio_k(t.size, c.meta["ratio"])
            assert topk_sets_match(t, idx, c[f"idx{s}"], k), (c.name, s)
            assert np.array_equal(np.sort(idx), np.sort(c[f"idx{s}"])), "random data has no ties"
            assert same_bits(res_new, c[f"res{s}"].ravel()), (c.name, s)
            assert same_bits(out, c[f"out{s}"].ravel()), (c.name, s)
            res = res_new


def test_randomk_golden(golden):
    for c in golden.cases("sparse", codec="randomk"):
        if "steps" in c.meta:
            continue
        # global_step is one counter per compressor instance, shared by all names
        step = c.meta["seed"] - sum(bytes(c.meta["name"], encoding="utf8"))
        idx, h = O.randomk_indices(c.meta["name"], step, c.meta["n"], c.meta["ratio"])
        assert h == c.meta["seed"]
        assert np.array_equal(idx, c["idx"]), c.name
        x = c["x"].ravel()
        assert same_bits(x[idx], c["vals"])
        assert same_bits(O.randomk_decode(x[idx], idx, x.size), c["dec"].ravel()), c.name


def test_randomk_allreduce_sequence(golden):
    c = golden.case("sparse", "randomk_residual_allreduce")
    res = None
    for s in range(2):
        t = O.residual_compensate(c[f"g{s}"], res).ravel()
        idx, h = O.randomk_indices("w", s, t.size, 0.1)
        assert h == int(c[f"seed{s}"][0])
        assert np.array_equal(idx, c[f"idx{s}"])
        dec = O.randomk_decode(t[idx], idx, t.size)
        res = O.residual_update(t, dec)
        assert same_bits(res, c[f"res{s}"].ravel())
        assert same_bits(dec, c[f"out{s}"].ravel())


def test_threshold_golden(golden):
    cases = golden.cases("sparse", codec="threshold")
    assert len(cases) >= 18
    for c in cases:
        x = c["x"].ravel()
        vals, idx = O.threshold_select(x, c.meta["threshold"])
        assert np.array_equal(idx, c["idx"]), c.name
        assert same_bits(vals, c["vals"]), c.name
        assert same_bits(O.sparse_decode(vals, idx, x.size), c["dec"].ravel()), c.name


# ----------------------------------------------------------------------------- quantisers
def test_terngrad_golden(golden):
    cases = golden.cases("quant", codec="terngrad")
    assert len(cases) >= 7
    for c in cases:
        codes, scalar = O.terngrad_compress(c["x"], c["u"])
        assert same_bits(scalar, c["scalar"].ravel()), c.name
        assert np.array_equal(codes, c["codes"].ravel()), c.name
        assert same_bits(O.terngrad_decode(codes, scalar), c["dec"].ravel()), c.name


def test_qsgd_golden(golden):
    cases = golden.cases("quant", codec="qsgd")
    assert len(cases) >= 30
    for c in cases:
        q, b = c.meta["quantum_num"], c.meta["bucket_size"]
        norms = O.qsgd_norms(c["x"], b)
        assert same_bits(norms, c["norms"]), c.name
        codes, _ = O.qsgd_compress(c["x"], c["u"], q, b)
        assert codes.dtype == c["codes"].dtype
        assert same_bits(codes, c["codes"].ravel()), c.name
        dec = O.qsgd_decode(codes, norms, q, b, c["x"].size)
        assert same_bits(dec, c["dec"].ravel()), c.name


def test_fp16_golden(golden):
    for c in golden.cases("quant", codec="fp16"):
        h = O.fp16_compress(c["x"])
        assert same_bits(h, c["half"]), c.name
        assert same_bits(O.fp16_decode(h), c["dec"]), c.name


# ----------------------------------------------------------------------------- natural (unpinned)
def test_natural_restatement_kat():
    """Parity unpinned (cupy absent): known-answer checks derived from natural.py:12-40."""
    x = np.array([1.0, -1.0, 0.0, 2.0 ** -109, 2.0 ** -110, 2.0 ** 18, 2.0 ** 19, 1.5, -0.75, np.inf],
                 dtype=np.float32)
    zero = np.zeros(x.size, dtype=np.int32)          # mantissa > 0 rounds up
    full = np.full(x.size, 0x7FFFFE, dtype=np.int32)  # never rounds up
    c_up = O.natural_compress(x, zero)
    c_dn = O.natural_compress(x, full)
    # 1.0 = 2^0: biased E = 127 -> code 109
    assert c_dn[0] == 109 and c_dn[1] == 128 + 109
    assert c_dn[2] == 0
    assert c_dn[3] == 0 and c_dn[4] == 0          # E' = 18 -> 0; below clips to 18 -> 0
    assert c_dn[5] == 127 and c_dn[6] == 127      # 2^18 -> E 145 -> 127 ; 2^19 clips
    assert c_up[7] == 110 and c_dn[7] == 109      # 1.5 rounds to 2 or 1
    assert c_dn[8] == 128 + 108
    dec = O.natural_decode(c_dn)
    assert dec[0] == 1.0 and dec[1] == -1.0 and dec[7] == 1.0 and dec[8] == -0.5
    assert dec[5] == 2.0 ** 18
    d0 = O.natural_decode(np.array([0, 128], dtype=np.uint8))
    assert same_bits(d0, np.array([0.0, -0.0], dtype=np.float32))


def test_cnat_restatement_kat():
    """Parity unpinned (CUDA only): cnat_cuda.cu LUT semantics, deterministic variant."""
    x = np.array([1.0, 0.75, -1.0, 0.0, 2.0 ** -109, 2.0 ** -110, 2.0 ** 20, -(2.0 ** -120)],
                 dtype=np.float32)
    c = O.cnat_compress(x)
    # 1.0 = 0.5*2^1: prob = 0 -> exp 0 -> biased 127 -> 110
    assert c[0] == 110
    # 0.75 = 0.75*2^0: prob 0.5 -> 0.5 >= 0.5 -> exp -1 -> biased 126 -> 109
    assert c[1] == 109
    assert c[2] == 128 + 110
    assert c[3] == 0
    assert c[4] == 1                 # 2^-109 = 0.5*2^-108 -> biased 18 -> code 1
    assert c[5] == 0                 # biased 17 -> 0
    assert c[6] == 127               # saturates
    assert c[7] == 128               # tiny negative
    d = O.cnat_decode(c)
    assert d[0] == 1.0 and d[1] == 0.5 and d[2] == -1.0 and d[3] == 0.0
    assert same_bits(d[7:8], np.array([-0.0], dtype=np.float32))


# ----------------------------------------------------------------------------- PowerSGD
def test_orthogonalize_golden(golden):
    for c in golden.cases("powersgd", codec="orthogonalize"):
        assert np.allclose(O.orthogonalize(c["a"]), c["out"], rtol=1e-5, atol=1e-6), c.name


def test_powersgd_golden(golden):
    for c in golden.cases("powersgd", codec="powersgd"):
        if "steps" in c.meta:
            continue
        x = c["x"]
        mat = x.reshape(x.shape[0], -1)
        p, q = O.powersgd_compress(mat, c["q0"])
        m = mat.shape[1]
        tol = 1e-5 * np.sqrt(m)
        assert np.allclose(p, c["p"], rtol=tol, atol=tol), c.name
        assert np.allclose(q, c["q"], rtol=tol, atol=tol * np.abs(c["q"]).max()), c.name
        dec = O.powersgd_decode(p, q)
        assert np.allclose(dec, c["dec"].reshape(dec.shape), rtol=tol, atol=tol * np.abs(c["dec"]).max())


def test_powersgd_memory_sequence(golden):
    c = golden.case("powersgd", "powersgd_memory_seq")
    res = None
    for s in range(2):
        g = c[f"g{s}"]
        t = g if res is None else (g + res).astype(np.float32)
        assert np.array_equal(t, c[f"t{s}"])
        q0 = O.orthogonalize(c[f"qdraw{s}"])
        p, q = O.powersgd_compress(t, q0)
        assert np.allclose(p, c[f"p{s}"], rtol=1e-4, atol=1e-5)
        dec = O.powersgd_decode(p, q)
        res = (t - dec).astype(np.float32)
        assert np.allclose(res, c[f"res{s}"], rtol=1e-4, atol=1e-4)


# ----------------------------------------------------------------------------- world 2
def test_world2_topk_aggregate(golden):
    r0, r1 = golden.case("world2", "rank0"), golden.case("world2", "rank1")
    res = [None, None]
    for s in range(2):
        decs, news = [], []
        for rank, c in enumerate((r0, r1)):
            t, vals, idx, new_res, _ = O.topk_residual_step(c[f"topk_g{s}"], res[rank], 0.01)
            assert np.array_equal(np.sort(idx), np.sort(c[f"topk_idx{s}"]))
            assert same_bits(new_res, c[f"topk_res{s}"])
            decs.append(O.sparse_decode(vals, idx, t.size))
            news.append(new_res)
        out = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
        for c in (r0, r1):
            assert same_bits(out, c[f"topk_out{s}"])
        res = news


def test_world2_sign_qsgd_terngrad(golden):
    r0, r1 = golden.case("world2", "rank0"), golden.case("world2", "rank1")
    agg = O.sign_aggregate([O.sign_decode(O.sign_encode(c["sign_g"])) for c in (r0, r1)])
    assert same_bits(agg, r0["sign_out"]) and same_bits(agg, r1["sign_out"])
    decs = []
    for c in (r0, r1):
        codes, norms = O.qsgd_compress(c["qsgd_g"], c["qsgd_u"], 127, 128)
        assert np.array_equal(codes, c["qsgd_codes"])
        decs.append(O.qsgd_decode(codes, norms, 127, 128, 4099))
    out = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
    assert same_bits(out, r0["qsgd_out"])
    decs = []
    for c in (r0, r1):
        codes, scalar = O.terngrad_compress(c["tern_g"], c["tern_u"])
        assert np.array_equal(codes, c["tern_codes"])
        decs.append(O.terngrad_decode(codes, scalar))
    out = (O.python_sum(decs) / np.float32(2)).astype(np.float32)
    assert same_bits(out, r0["tern_out"])


def test_world2_randomk_allreduce(golden):
    r0, r1 = golden.case("world2", "rank0"), golden.case("world2", "rank1")
    # same seed on both ranks -> same indices; Allreduce sums values then /W
    assert np.array_equal(r0["randk_idx"], r1["randk_idx"])
    idx = r0["randk_idx"].astype(np.int64)
    vals = ((r0["randk_g"].ravel()[idx] + r1["randk_g"].ravel()[idx]) / np.float32(2)).astype(np.float32)
    out = O.randomk_decode(vals, idx, 4099)
    assert same_bits(out, r0["randk_out"].ravel())


def test_dgc_oracle_vs_reference(golden):
    cases = golden.cases("dgc", codec="dgc")
    assert cases
    for c in cases:
        vals, idx, mask, _ = O.dgc_compress(c["x"], c["sample_idx"], c.meta["ratio"])
        assert np.array_equal(idx, c["idx"]), c.name
        assert same_bits(vals, c["vals"]), c.name
        assert np.array_equal(mask.astype(np.uint8), c["mask"].ravel()), c.name
        assert same_bits(O.sparse_decode(vals, idx, c["x"].size), c["dec"].ravel()), c.name


def test_dgc_memory_oracle_vs_reference(golden):
    for c in golden.cases("dgc", codec="dgc_memory"):
        r = a = None
        for s in range(c.meta["steps"]):
            t, r, a = O.dgc_memory_compensate(c[f"g{s}"], r, a, c.meta["momentum"])
            assert same_bits(t, c[f"t{s}"]), (c.name, s)
            vals, idx, mask, _ = O.dgc_compress(t, c[f"sidx{s}"], c.meta["ratio"])
            assert np.array_equal(idx, c[f"idx{s}"]) and same_bits(vals, c[f"vals{s}"]), (c.name, s)
            r, a = O.dgc_memory_update(r, a, mask)
            assert same_bits(r, c[f"res{s}"]) and same_bits(a, c[f"grad{s}"]), (c.name, s)
    quirk = golden.case("dgc", "dgc_clipping_quirk")
    assert bool(quirk["flag"][0])   # the reference's gradient_clipping=True raises TypeError


# ----------------------------------------------------------------------------- Horovod flavour
def test_torchflav_qsgd_global_norm(golden):
    cases = golden.cases("torchflav", codec="qsgd")
    assert len(cases) >= 14
    for c in cases:
        q = c.meta["quantum_num"]
        codes, norm = O.qsgd_global_compress(c["x"], c["u"], q)
        assert same_bits(norm, c["norm"].ravel()), c.name
        assert same_bits(codes, c["codes"].ravel()), c.name
        assert same_bits(O.qsgd_global_decode(c["codes"].ravel(), c["norm"], q, c["x"].size), c["dec"].ravel()), c.name


def test_torchflav_threshold_strict(golden):
    for c in golden.cases("torchflav", codec="threshold"):
        v, i = O.threshold_select_strict(c["x"], c.meta["threshold"])
        assert np.array_equal(i, c["idx"]), c.name
        assert same_bits(v, c["vals"]), c.name


def test_torchflav_randomk_randperm(golden):
    for c in golden.cases("torchflav", codec="randomk"):
        idx, h = O.randomk_perm_indices(c.meta["name"], c.meta["seed"] - sum(bytes(c.meta["name"], "utf8")),
                                        c.meta["n"], c.meta["ratio"])
        assert h == c.meta["seed"]
        assert np.array_equal(idx, c["idx"]), c.name
        assert np.unique(idx).size == idx.size


def test_torchflav_topk_int64(golden):
    for c in golden.cases("torchflav", codec="topk"):
        assert c["idx"].dtype == np.int64
        k = O.ratio_k(c["x"].size, c.meta["ratio"])
        v, i = O.topk_select(c["x"].ravel(), k)
        assert topk_sets_match(c["x"].ravel(), i, c["idx"], k), c.name


def test_torchflav_terngrad_equals_dist_rule(golden):
    """uniform_(0, scalar) (torch flavour) == uniform_(0, 1) * scalar (dist flavour), bit for bit."""
    for c in golden.cases("torchflav", codec="terngrad"):
        codes, scal = O.terngrad_compress(c["x"], c["u"])
        assert np.array_equal(codes, c["codes"].ravel()), c.name
        assert same_bits(scal, c["scalar"].ravel()), c.name
        assert same_bits(O.terngrad_decode(codes, scal), c["dec"].ravel()), c.name
