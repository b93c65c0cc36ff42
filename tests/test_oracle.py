"""CPU tests of the oracle (the checker) against the reference's own code and
tests: the compiled estimate stage (oracle/_ref, build container only), the
committed fixtures, and the reference's known-answer tests."""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from conftest import golden

FIXTURES = ["ndt_U4096_k256_s0.npz", "ndt_U4096_k256_s1.npz", "ndt_L4096_k256_s0.npz", "ndt_L4096_k256_s1.npz",
            "ndt_U2003_k128_s7.npz"]


def test_limits_kat():
    """core_legacy/tests/test_pointclouds.cpp:5-24 (and the 30-point variant
    called with num_points = 6, :25-68): max/min of a 6-point cloud."""
    cloud = np.array([[0, 1, 0], [1, 0, 0], [0, -1, 0], [-1, 0, 0], [0, 0, 1], [0, 0, -2]], dtype=np.float64)
    lim = np.zeros(6)
    O.lib().orc_limits(O._ptr(cloud), 3, ctypes.c_uint64(6), O._ptr(lim))
    assert list(lim) == [1.0, 1.0, 1.0, -1.0, -1.0, -2.0]
    five = np.tile(cloud, (5, 1))
    O.lib().orc_limits(O._ptr(five), 3, ctypes.c_uint64(6), O._ptr(lim))
    assert list(lim) == [1.0, 1.0, 1.0, -1.0, -1.0, -2.0]


def test_limits_dbl_min_quirk():
    """max starts at DBL_MIN (pointclouds.c:44-46): an all-negative axis keeps it."""
    cloud = -np.abs(np.random.default_rng(0).normal(size=(50, 3))) - 1
    lim = np.zeros(6)
    O.lib().orc_limits(O._ptr(cloud), 3, ctypes.c_uint64(50), O._ptr(lim))
    assert lim[0] == lim[1] == lim[2] == np.finfo(np.float64).tiny


def rand_clouds(loops=10, n=90000):
    buf = np.zeros(n * 3)
    for i in range(loops):
        O.lib().orc_glibc_rand_points(O._ptr(buf), ctypes.c_uint64(n * 3), ctypes.c_uint(0), ctypes.c_int(i == 0))
        yield buf.reshape(n, 3).copy()


def test_reference_smoke_ndt_downsample():
    """core_legacy/tests/ndt_downsample.c: 10 x ndt_downsample of 90k rand()
    points to 24 NDs must return 0."""
    for pts in rand_clouds():
        r = O.run(pts, 24)
        assert r.rc == 0 and r.nout == 24


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference_fixtures(name):
    z = golden(name)
    pts = z["points"].astype(np.float64)
    k = int(z["k"])
    r = O.run(pts, k, classes=z["labels"], num_classes=int(z["num_classes"]))
    assert r.rc == 0
    assert np.array_equal(r.search.guesses, z["ref_guesses"])
    assert np.array_equal(r.search.counts, z["ref_counts"])
    assert tuple(r.search.len) == tuple(z["ref_len"])
    assert np.array_equal(r.vox_n, z["ref_count"])
    assert np.array_equal(r.vox_mean, z["ref_mean"])
    assert np.array_equal(r.vox_cov_pre, z["ref_cov"])
    occ = z["ref_count"] > 0
    assert np.array_equal(r.vox_cls[occ], z["ref_cls"][occ])
    # stages past the estimate are the oracle's own (regression pins)
    assert np.array_equal(r.ord_div, z["orc_ord_div"], equal_nan=True)
    assert np.array_equal(r.vox_kept, z["orc_kept"])
    assert np.array_equal(r.out_cov, z["orc_out_cov"], equal_nan=True)


@pytest.mark.skipif(not os.path.exists(O.REF_LIB), reason="oracle/_ref is built only where /root/reference exists")
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_matches_live_reference(seed):
    """Live comparison with the reference's compiled estimate stage, including
    an abandoned chunk (a point exactly on the grid maximum)."""
    from ndnet.synthetic import lidar_cloud, uniform_cloud
    rng = np.random.default_rng(seed)
    clouds = [uniform_cloud(20_000 + seed, seed).astype(np.float64), lidar_cloud(20_003, seed).astype(np.float64)]
    a = rng.uniform(0.0, 14.995, (4101, 3))
    a[17] = [14.995, 3.0, 3.0]
    a[1000] = [0.0, 0.0, 0.0]
    clouds.append(a)
    for pts in clouds:
        for k in (64, 300):
            r = O.run(pts, k)
            rc, g, c, ln, off, vs = O.ref_search(pts, k)
            assert rc == r.rc
            assert np.array_equal(g, r.search.guesses) and np.array_equal(c, r.search.counts)
            if rc == 0:
                cnt, mean, cov, _, _ = O.ref_estimate(pts, vs, ln, off)
                assert np.array_equal(cnt, r.vox_n)
                assert np.array_equal(mean, r.vox_mean)
                assert np.array_equal(cov, r.vox_cov_pre)


@pytest.mark.skipif(not os.path.exists(O.REF_LIB), reason="needs oracle/_ref")
def test_reference_threads_counts_and_means():
    """The shipped 8-thread estimate: counts equal, means within rounding
    (its off-diagonals depend on thread interleaving)."""
    pts = golden("ndt_U4096_k256_s0.npz")["points"].astype(np.float64)
    r = O.run(pts, 256)
    cnt, mean, cov, _, _ = O.ref_estimate(pts, r.search.voxel_size, r.search.len, r.search.off, threads=True)
    assert np.array_equal(cnt, r.vox_n)
    assert np.allclose(mean, r.vox_mean, rtol=0, atol=1e-12)
    d = np.arange(9) % 4 == 0
    assert np.allclose(cov[:, d], r.vox_cov_pre[:, d], rtol=1e-12, atol=1e-14)


def test_portable_log_correctly_rounded():
    import decimal
    decimal.getcontext().prec = 50
    rng = np.random.default_rng(1)
    x = np.concatenate([np.exp(rng.uniform(-700, 700, 3000)), rng.uniform(0.5, 2.0, 3000),
                        1 + rng.normal(0, 1e-9, 500), [1.0, 2.0, 0.5, 1e-310, 5e-324, 1.7976931348623157e308]])
    y = np.zeros_like(x)
    g = np.zeros_like(x)
    O.lib().orc_portable_log_many(O._ptr(x), O._ptr(y), ctypes.c_uint64(len(x)))
    O.lib().orc_libm_log_many(O._ptr(x), O._ptr(g), ctypes.c_uint64(len(x)))
    cr = np.array([float(decimal.Decimal(float(v)).ln()) for v in x])
    assert (y != cr).sum() == 0
    assert (np.abs(y - g) <= np.spacing(np.abs(g))).all()  # within 1 ulp of glibc
    assert np.isneginf(O.lib().orc_portable_log(0.0)) and np.isnan(O.lib().orc_portable_log(-1.0))


def test_portable_log_keeps_kept_sets():
    """glibc log vs the portable log: identical pruned sets on the fixtures."""
    for name in FIXTURES:
        z = golden(name)
        assert np.array_equal(z["orc_kept"], z["orc_glibc_kept"])


def test_prune_walk_quirks():
    """prune_nds bound check against the decremented count, and the -1 path."""
    from ndnet.synthetic import uniform_cloud
    pts = uniform_cloud(4096, 0).astype(np.float64)
    ch = O.LegacyChain(pts)
    ch.downsample(256)
    assert ch.rc == 0
    nkl0 = ch.nkl.value
    ch.prune(300)  # more than valid -> -1, nothing changes
    assert ch.rc == -1 and ch.nvalid.value == 256 and ch.nkl.value == nkl0
    ch.prune(128)
    assert ch.rc == 0 and ch.nvalid.value == 128 and ch.nkl.value == nkl0 - 128
    ch.cleanup()


def _lu_invert(A, variant):
    A = np.ascontiguousarray(A, dtype=np.float64)
    LU, perm, inv = np.zeros(9), np.zeros(3, np.int32), np.zeros(9)
    O.lib().orc_lu_invert_test(O._ptr(A), O._ptr(LU), O._ptr(perm), O._ptr(inv), ctypes.c_int(variant))
    return inv.reshape(3, 3), LU.reshape(3, 3), perm


def test_gsl_lu_invert_restatement():
    """gsl_linalg_LU_invert as GSL 2.7.1 publishes it (tri_invert U, tri_invert
    L unit, tri_UL, inverse column permutation; kullback_leibler.c:92): an
    inverse to rounding, its permutation handling exact, and a rounding
    sequence of its own (it differs in the last bits from the column-solve
    variant round 1 used)."""
    rng = np.random.default_rng(0)
    differs = 0
    for _ in range(2000):
        A = rng.normal(size=(3, 3))
        g, _, _ = _lu_invert(A, 1)
        c, _, _ = _lu_invert(A, 0)
        ref = np.linalg.inv(A)
        assert np.abs(g - ref).max() <= 1e-11 * np.abs(ref).max()
        differs += not np.array_equal(g, c)
    assert differs > 1000
    # a pure permutation with exact entries: exact inverse, and U^-1 L^-1 by hand
    P = 2.0 * np.array([[0, 1, 0], [0, 0, 1], [1, 0, 0]], dtype=np.float64)
    g, _, perm = _lu_invert(P, 1)
    assert np.array_equal(g, P.T / 4.0)
    A = np.array([[4.0, 3.0, 2.0], [2.0, 1.0, 3.0], [3.0, 2.0, 1.0]])
    g, LU, perm = _lu_invert(A, 1)
    U, L = np.triu(LU), np.tril(LU, -1) + np.eye(3)
    Pm = np.zeros((3, 3))
    Pm[np.arange(3), perm] = 1.0
    assert np.allclose(Pm @ A, L @ U, rtol=0, atol=1e-15)
    assert np.allclose(g, np.linalg.inv(U) @ np.linalg.inv(L) @ Pm, rtol=1e-15, atol=1e-15)


def test_fullsize_fixture_pins_oracle():
    """The oracle still produces the committed full-size digests (one cloud of
    each C2 / C5 case; tests/golden/make_fullsize.py)."""
    import hashlib
    from ndnet.synthetic import make_batch
    z = golden("fullsize_rows.npz")
    for cfg, clouds in (("C2", (("U", 3), ("L", 5))), ("C5", (("U", 3), ("L", 5))), ("C4", (("U", 101), ("L", 77)))):
        levels = [int(v) for v in z[f"levels_{cfg}"]]
        for kind, b in clouds:
            pts = make_batch(kind, 1, int(z["points"]), seed0=b)[0].astype(np.float64)
            ch = O.LegacyChain(pts)
            res = [ch.downsample(levels[0])] + [ch.prune(k) for k in levels[1:]]
            ch.cleanup()
            for lv, (pc, cov) in enumerate(res):
                rows = np.zeros((len(pc), 12), np.float32)
                rows[:, :3] = np.nan_to_num(pc.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
                rows[:, 3:] = np.nan_to_num(cov.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
                assert hashlib.sha256(rows.tobytes()).digest() == z[f"{cfg}_{kind}_sha"][b, lv].tobytes()


def test_rtab_division_is_ieee():
    """k_welford_q's long-ND path divides t / n as fma(t, rc, t * rl)
    (csrc/ndt_kernels.hip, wq_heavy): bit-identical to the IEEE division on
    10^7 random operands over the range its fast path admits, n up to 2^22
    plus powers of two and their neighbours."""
    import ctypes
    L = O.lib()
    L.orc_rtab_div_mismatches.restype = ctypes.c_uint64
    L.orc_rtab_div_mismatches.argtypes = [ctypes.c_uint64] * 3
    assert L.orc_rtab_div_mismatches(1 << 22, 10_000_000, 7) == 0
