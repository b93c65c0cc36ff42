"""Parity of the HIP NDT path with the CPU oracle and the reference fixtures.

Bar: bit-exact for integer/index results (grid, counts, dense order, KL list
order, kept set) and for every double the reference computes (means,
covariances, KL scores: the kernels perform the same IEEE operations);
float32 rows equal the oracle's after the same cast + nan_to_num.
"""
import ctypes

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

FIXTURES = ["ndt_U4096_k256_s0.npz", "ndt_U4096_k256_s1.npz", "ndt_L4096_k256_s0.npz", "ndt_L4096_k256_s1.npz",
            "ndt_U2003_k128_s7.npz"]


def _run_plan(points_b: np.ndarray, k: int, labels_b=None, num_classes=-1, exact_counts=True):
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    B, n, _ = points_b.shape
    plan = NdtPlan(B, n, k, num_classes)
    plan.set_exact_counts(exact_counts)
    pts = torch.from_numpy(np.ascontiguousarray(points_b, dtype=np.float32)).cuda()
    lbl = None if labels_b is None else torch.from_numpy(labels_b.astype(np.int32)).cuda()
    out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
    out_cls = None if labels_b is None else torch.empty((B, k, num_classes + 1), dtype=torch.float32, device="cuda")
    plan.run(pts, lbl, out, out_cls)
    torch.cuda.synchronize()
    return plan, out.cpu().numpy(), (None if out_cls is None else out_cls.cpu().numpy())


def _dump(plan, cloud: int, nd: int, ne: int):
    from ndnet import _lib
    d = dict(nd_n=np.zeros(nd, np.uint32), nd_mean=np.zeros((nd, 3)), nd_cov_pre=np.zeros((nd, 9)),
             nd_cov_post=np.zeros((nd, 9)), vox=np.zeros(nd, np.uint32), ord_val=np.zeros(max(ne, 1)),
             ord_p=np.zeros(max(ne, 1), np.uint32), ord_q=np.zeros(max(ne, 1), np.uint32),
             guesses=np.zeros(16), counts=np.zeros(16, np.uint32), alive=np.zeros(nd, np.uint8))
    iters = ctypes.c_uint32(0)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = _lib.lib().ndnet_ndt_debug_dump(plan.handle, cloud, p(d["nd_n"]), p(d["nd_mean"]), p(d["nd_cov_pre"]),
                                         p(d["nd_cov_post"]), p(d["vox"]), p(d["ord_val"]), p(d["ord_p"]),
                                         p(d["ord_q"]), p(d["guesses"]), p(d["counts"]), ctypes.byref(iters),
                                         p(d["alive"]))
    assert rc == 0
    d["iters"] = iters.value
    return d


def _f32_rows(pc64, cov64, k):
    rows = np.zeros((k, 12), np.float32)
    rows[:, :3] = np.nan_to_num(pc64.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
    rows[:, 3:] = np.nan_to_num(cov64.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
    return rows


@pytest.mark.parametrize("name", FIXTURES)
def test_stages_match_reference_and_oracle(name):
    z = golden(name)
    k = int(z["k"])
    ncls = int(z["num_classes"])
    plan, out, out_cls = _run_plan(z["points"][None], k, z["labels"][None], ncls)
    st = plan.host_stats()[0]
    assert st.rc == 0 and st.prune_rc == int(z["orc_prune_rc"])
    # bisection: every guess and count of the reference's own estimate stage
    occ = np.nonzero(z["ref_count"])[0]
    nd = len(occ)
    d = _dump(plan, 0, nd, int(st.num_events))
    assert d["iters"] == len(z["ref_guesses"])
    assert np.array_equal(d["guesses"][:d["iters"]], z["ref_guesses"])
    assert np.array_equal(d["counts"][:d["iters"]], z["ref_counts"])
    assert tuple(st.len) == tuple(z["ref_len"]) and st.voxel_size == float(z["ref_voxel_size"])
    # per-ND state at the accepted size, dense ids in ascending voxel order
    assert st.num_nds == nd
    assert np.array_equal(d["vox"], occ)
    assert np.array_equal(d["nd_n"], z["ref_count"][occ])
    assert np.array_equal(d["nd_mean"], z["ref_mean"][occ])
    assert np.array_equal(d["nd_cov_pre"], z["ref_cov"][occ])
    # KL list in the reference's insertion order (oracle), prune, mutated covariances
    dense = -np.ones(len(z["ref_count"]) + 1, np.int64)
    dense[occ] = np.arange(nd)
    dense[-1] = 0xFFFFFFFF  # index -1: an entry the reference never wrote (poison)
    E = len(z["orc_ord_div"])
    assert st.num_events == E and st.num_kl == int(z["orc_post_nkl"])
    # the retained list after the level-1 prune's left shift (ndt.c:69-72)
    live = z["orc_post_p"] >= 0
    assert np.array_equal(d["ord_val"][:E][live], z["orc_post_div"][live], equal_nan=True)
    assert np.array_equal(d["ord_p"][:E], dense[z["orc_post_p"]])
    assert np.array_equal(d["ord_q"][:E], dense[z["orc_post_q"]])
    assert np.array_equal(d["nd_cov_post"], z["orc_cov_post"][occ], equal_nan=True)
    assert np.array_equal(d["alive"], z["orc_kept"][occ])
    assert st.num_out == int(z["orc_nout"]) and st.num_valid == int(z["orc_num_valid"])
    # rows as ndt_preprocessing returns them
    assert np.array_equal(out[0], _f32_rows(z["orc_out_pc"], z["orc_out_cov"], k))
    onehot = np.zeros((k, ncls + 1), np.float32)
    onehot[np.arange(k), z["orc_out_cls"]] = 1.0
    assert np.array_equal(out_cls[0], onehot)


@pytest.mark.parametrize("name", FIXTURES[:3])
def test_skipped_grids_change_nothing(name):
    """Default mode: grids with fewer voxels than k are not counted (their
    bisection decision, hi = guess, needs no count).  Same guesses, same
    counted counts, same outputs and stats as counting every grid; a count is
    skipped only where the grid has fewer than k voxels."""
    z = golden(name)
    k = int(z["k"])
    runs = {}
    for exact in (True, False):
        plan, out, _ = _run_plan(z["points"][None], k, exact_counts=exact)
        st = plan.host_stats()[0]
        d = _dump(plan, 0, int(st.num_nds), int(st.num_events))
        runs[exact] = (out, bytes(st), d)
    (o1, s1, d1), (o0, s0, d0) = runs[True], runs[False]
    assert np.array_equal(o1, o0) and s1 == s0
    it = d1["iters"]
    assert d0["iters"] == it and np.array_equal(d0["guesses"][:it], d1["guesses"][:it])
    skipped = d0["counts"][:it] == 0xFFFFFFFF
    assert skipped.any()
    assert np.array_equal(d0["counts"][:it][~skipped], d1["counts"][:it][~skipped])
    lim = z["points"].astype(np.float64)
    ext = lim.max(0) - lim.min(0)
    for g, sk in zip(d1["guesses"][:it], skipped):
        V = int(np.prod(np.ceil(ext / g)))
        assert sk == (V < k)


@pytest.mark.parametrize("kind", ["U", "L"])
def test_lazy_list_equals_eager(kind):
    """Lazy retained list (default): clouds with num_nds <= k score and sort
    no events in the run; a later prune level or dump builds the list on
    demand.  Rows, stats, every dumped intermediate (the list entry for
    entry) and two further prune levels equal the eager build's, bit for
    bit.  U at k = 1000 has num_nds = k in every cloud (the deferred case),
    L has num_nds > k (the list is built in the run either way)."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    B, n, k = 4, 100_000, 1000
    pts = torch.from_numpy(make_batch(kind, B, n)).cuda()
    res = {}
    for variant in ("eager", "lazy", "lazy_no_dump"):  # the last builds the list inside prune
        plan = NdtPlan(B, n, k, -1)
        plan.set_lazy_list(variant != "eager")
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        plan.run(pts, None, out, None)
        torch.cuda.synchronize()
        stats = plan.host_stats()
        if kind == "U":
            assert all(s.num_nds == k for s in stats)
        dumps = None
        if variant != "lazy_no_dump":
            dumps = [_dump(plan, b, int(stats[b].num_nds), int(stats[b].num_events)) for b in range(B)]
        levels = []
        for k2 in (600, 300):
            o2 = torch.empty((B, k2, 12), dtype=torch.float32, device="cuda")
            plan.prune(k2, o2)
            torch.cuda.synchronize()
            levels.append((o2.cpu().numpy(), [bytes(s) for s in plan.host_stats()]))
        res[variant] = (out.cpu().numpy(), [bytes(s) for s in stats], dumps, levels)
    o0, s0, d0, l0 = res["eager"]
    for variant in ("lazy", "lazy_no_dump"):
        o1, s1, d1, l1 = res[variant]
        assert np.array_equal(o0, o1) and s0 == s1, variant
        if d1 is not None:
            for b in range(B):
                for key in d0[b]:
                    assert np.array_equal(d0[b][key], d1[b][key], equal_nan=True), (b, key)
        for (a0, t0), (a1, t1) in zip(l0, l1):
            assert np.array_equal(a0, a1) and t0 == t1, variant


def test_reference_driver_fixture():
    """Rows the reference's own ndt_preprocessing produced (over the oracle ABI)."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    z = golden("preproc_B3_k256.npz")
    p, c, cl = ndt_preprocessing(int(z["k"]), torch.from_numpy(z["points"]).cuda())
    assert cl is None
    assert np.array_equal(p.cpu().numpy(), z["out_points"])
    assert np.array_equal(c.cpu().numpy(), z["out_covs"])


@pytest.mark.parametrize("kind", ["U", "L"])
def test_full_size_batch(kind):
    """C2: 16 x 100k -> 1000, every cloud against the oracle."""
    import torch
    import oracle as O
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing, last_stats
    from ndnet.synthetic import make_batch
    B, n, k = 16, 100_000, 1000
    pts = make_batch(kind, B, n)
    p, c, _ = ndt_preprocessing(k, torch.from_numpy(pts).cuda())
    p, c = p.cpu().numpy(), c.cpu().numpy()
    stats = last_stats()
    for b in range(B):
        pc, cov, r = O.downsample_f32(pts[b], k)
        assert stats[b].rc == r.rc == 0
        assert stats[b].num_events == len(r.ord_div)
        assert np.array_equal(p[b], pc), f"cloud {b} means"
        assert np.array_equal(c[b], cov), f"cloud {b} covariances"


def test_mixed_batch_equals_single_runs():
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing
    names = FIXTURES[:4]
    pts = np.stack([golden(nm)["points"] for nm in names])
    p, c, _ = ndt_preprocessing(256, torch.from_numpy(pts).cuda())
    for b, nm in enumerate(names):
        z = golden(nm)
        rows = _f32_rows(z["orc_out_pc"], z["orc_out_cov"], 256)
        assert np.array_equal(p[b].cpu().numpy(), rows[:, :3])
        assert np.array_equal(c[b].cpu().numpy(), rows[:, 3:])


def test_edge_clouds():
    """A failed search (z constant and positive: a 0-length axis puts every
    point out of grid), and a cloud whose extent is exactly one first-pass
    voxel, so a reference worker abandons the rest of its chunk at the point on
    the grid maximum (float64 path: the extent is not float32-representable)."""
    import torch
    import oracle as O
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.preprocessing.ndt_legacy import NDT_Sampler
    rng = np.random.default_rng(5)
    n, k = 4101, 200
    flat = rng.uniform(-5, 5, (n, 3)).astype(np.float32)
    flat[:, 2] = 1.5
    plan = NdtPlan(1, n, k, -1)
    out = torch.full((1, k, 12), 7.0, dtype=torch.float32, device="cuda")
    plan.run(torch.from_numpy(flat[None]).cuda(), None, out, None)
    torch.cuda.synchronize()
    st = plan.host_stats()[0]
    r = O.run(flat.astype(np.float64), k)
    assert st.rc == r.rc == -3 and st.iters == 15
    assert not out.any().item()
    # abandoned chunks
    a = rng.uniform(0.0, 14.995, (n, 3))
    a[17] = [14.995, 3.0, 3.0]
    a[1000] = [0.0, 0.0, 0.0]
    assert (a[:, 0].max() - a[:, 0].min()) / 14.995 == 1.0
    s = NDT_Sampler(a)
    pc, cov, _ = s.downsample(k)
    ref = O.LegacyChain(a)
    pc2, cov2 = ref.downsample(k)
    assert np.array_equal(pc, pc2) and np.array_equal(cov, cov2, equal_nan=True)
    s.cleanup()
    ref.cleanup()


def test_legacy_sampler_multilevel():
    """NDT_Sampler.downsample(k) -> prune(k2) -> prune(k3) (config 5's levels)
    against the oracle's implementation of the same reference ABI calls."""
    import oracle as O
    from ndnet.preprocessing.ndt_legacy import NDT_Sampler
    from ndnet.synthetic import uniform_cloud, lidar_cloud
    for cloud in (uniform_cloud(30_000, 3), lidar_cloud(30_000, 4)):
        pts = cloud.astype(np.float64)
        s = NDT_Sampler(pts)
        levels = [s.downsample(600), s.prune(300), s.prune(150)]
        ref = O.LegacyChain(pts)
        expect = [ref.downsample(600), ref.prune(300), ref.prune(150)]
        for (p1, c1, _), (p2, c2) in zip(levels, expect):
            assert np.array_equal(p1, p2)
            assert np.array_equal(c1, c2, equal_nan=True)
        # the reference's class dtypes: uint16 from downsample (ndt_legacy.py:138),
        # int16 from prune (:211)
        assert [lv[2].dtype for lv in levels] == [np.uint16, np.int16, np.int16]
        s.cleanup()
        ref.cleanup()


def _wide_sparse(n, seed):
    """Most points in a small box, a few far outliers: the early bisection
    grids exceed the 32768-voxel bitmap and run through the per-voxel stamps."""
    rng = np.random.default_rng(seed)
    a = rng.uniform(-3, 3, (n, 3))
    a[::997] = rng.uniform(-40, 40, (len(a[::997]), 3))
    return a.astype(np.float32)


@pytest.mark.parametrize("case", ["U", "L", "wide", "mixed"])
def test_front_kernel_equals_multikernel_path(case):
    """k_front (one launch: limits, bisection, dense ids, binning) against the
    one-launch-per-stage path on the same batch: every output row, every
    stats field and every intermediate the dump exposes, bit for bit; both
    are also checked against the oracle."""
    import torch
    import oracle as O
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    if case == "wide":
        pts = np.stack([_wide_sparse(30_000, s) for s in range(3)])
        k = 300
    elif case == "mixed":
        pts = np.stack([make_batch("U", 1, 30_000, seed0=5)[0], make_batch("L", 1, 30_000, seed0=6)[0],
                        _wide_sparse(30_000, 9)])
        k = 300
    else:
        pts = make_batch(case, 5, 50_000, seed0=21)
        k = 700
    B, n, _ = pts.shape
    res = {}
    for path in (1, 2):
        plan = NdtPlan(B, n, k, -1)
        plan.set_path(path)
        plan.set_exact_counts(True)
        assert plan.path == path
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        plan.run(torch.from_numpy(pts).cuda(), None, out, None)
        torch.cuda.synchronize()
        stats = plan.host_stats()
        dumps = [_dump(plan, b, int(stats[b].num_nds), int(stats[b].num_events)) for b in range(B)]
        res[path] = (out.cpu().numpy(), stats, dumps)
    o1, s1, d1 = res[1]
    o2, s2, d2 = res[2]
    assert np.array_equal(o1, o2)
    for b in range(B):
        assert bytes(s1[b]) == bytes(s2[b]), f"cloud {b} stats"
        for key in d1[b]:
            assert np.array_equal(d1[b][key], d2[b][key], equal_nan=True), (b, key)
        pc, cov, r = O.downsample_f32(pts[b], k)
        assert s2[b].rc == r.rc
        if r.rc == 0:
            assert np.array_equal(o2[b, :, :3], pc) and np.array_equal(o2[b, :, 3:], cov)


@pytest.mark.parametrize("vcap", [40, 120, 900, 6000])
def test_voxel_capacity_overflow_paths_agree(vcap):
    """A grid of more voxels than the plan's capacity fails the cloud (rc -1,
    the reference's malloc of V NDs) at the iteration it appears: on a grid
    too small to count (k_front's skipped iterations, run as lanes of one
    wave) or on a counted one.  k_front and the one-launch-per-stage path
    agree on every stats field, and U's clouds reach both kinds."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    pts = np.concatenate([make_batch("U", 2, 20_000, seed0=3), make_batch("L", 1, 20_000, seed0=4)])
    B, n, _ = pts.shape
    k = 300
    res = {}
    for path in (1, 2):
        plan = NdtPlan(B, n, k, -1, voxel_capacity=vcap)
        plan.set_path(path)
        assert plan.path == path
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        plan.run(torch.from_numpy(pts).cuda(), None, out, None)
        torch.cuda.synchronize()
        res[path] = (out.cpu().numpy(), plan.host_stats())
    for b in range(B):
        assert bytes(res[1][1][b]) == bytes(res[2][1][b]), f"cloud {b} stats (vcap {vcap})"
    assert np.array_equal(res[1][0], res[2][0])
    if vcap == 40:  # overflows while the grids are still too small to count
        assert all(st.rc == -1 for st in res[2][1])


@pytest.mark.parametrize("kind", ["U", "L"])
def test_multiscale_batch_matches_oracle_chain(kind):
    """Config C5's path batched: downsample(600) -> prune(300) -> prune(150)
    for 4 clouds at once (ndt_multiscale), every level's rows bit-exact
    against the oracle's downsample/prune_nds/to_point_cloud chain per cloud
    after the driver's float32 cast and nan_to_num."""
    import oracle as O
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_multiscale
    from ndnet.synthetic import make_batch
    pts = make_batch(kind, 4, 30_000, seed0=11)
    levels = ndt_multiscale((600, 300, 150), torch.from_numpy(pts).cuda())
    f32 = lambda a: np.nan_to_num(a.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)  # noqa: E731
    for b in range(4):
        ref = O.LegacyChain(pts[b].astype(np.float64))
        expect = [ref.downsample(600), ref.prune(300), ref.prune(150)]
        for (p, c, _), (p2, c2) in zip(levels, expect):
            assert np.array_equal(p[b].cpu().numpy(), f32(p2))
            assert np.array_equal(c[b].cpu().numpy(), f32(c2))
        ref.cleanup()


@pytest.mark.parametrize("kind", ["U", "L"])
def test_c5_full_size_levels(kind):
    """Config C5 as configured (BASELINE.json config 5): 16 x 100k points ->
    downsample(2000) -> prune(1000) -> prune(500), batched on the GPU
    (ndt_multiscale), every level of every cloud bit-exact against the
    oracle's NDT_Sampler chain (ndt_legacy.py:111-240: ndt_downsample, then
    prune_nds + to_point_cloud on the retained KL list)."""
    import oracle as O
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_multiscale
    from ndnet.synthetic import make_batch
    B, n, levels = 16, 100_000, (2000, 1000, 500)
    pts = make_batch(kind, B, n)
    out = ndt_multiscale(levels, torch.from_numpy(pts).cuda())
    got = [(p.cpu().numpy(), c.cpu().numpy()) for p, c, _ in out]
    f32 = lambda a: np.nan_to_num(a.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)  # noqa: E731
    for b in range(B):
        ref = O.LegacyChain(pts[b].astype(np.float64))
        expect = [ref.downsample(levels[0])] + [ref.prune(k) for k in levels[1:]]
        assert ref.rc == 0
        for lv, ((p, c), (p2, c2)) in enumerate(zip(got, expect)):
            assert np.array_equal(p[b], f32(p2)), f"cloud {b} level {lv} means"
            assert np.array_equal(c[b], f32(c2)), f"cloud {b} level {lv} covariances"
        ref.cleanup()


def test_check_flag_raises_on_failed_cloud():
    """opt-in failure check (the reference ignores return codes)."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtCloudError, ndt_preprocessing
    rng = np.random.default_rng(2)
    pts = rng.uniform(-5, 5, (2, 4096, 3)).astype(np.float32)
    pts[1, :, 2] = 1.5  # a zero-length axis: the search reaches 15 iterations (-3)
    t = torch.from_numpy(pts).cuda()
    p, c, _ = ndt_preprocessing(200, t)  # default: zero rows, like the reference
    assert not p[1].any().item() and p[0].any().item()
    with pytest.raises(NdtCloudError) as ei:
        ndt_preprocessing(200, t, check=True)
    assert ei.value.rcs == [0, -3]


def _sha_rows(a) -> bytes:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).digest()


@pytest.mark.parametrize("cfg,kind", [("C2", "U"), ("C2", "L"), ("C5", "U"), ("C5", "L")])
def test_fullsize_fixture(cfg, kind):
    """Configs C2 and C5 at full size against the committed full-size fixture
    (tests/golden/make_fullsize.py): every cloud's float32 rows at every level
    hash-equal to the oracle's canonical variant (portable log + GSL 2.7.1
    LU_invert).  The fixture also records, per cloud and level, how many kept
    NDs the glibc-log and column-inverse variants change: zero everywhere at
    these sizes, so the HIP rows equal those variants' too."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_multiscale
    from ndnet.synthetic import make_batch
    z = golden("fullsize_rows.npz")
    B, n = int(z["batch"]), int(z["points"])
    levels = tuple(int(v) for v in z[f"levels_{cfg}"])
    out = ndt_multiscale(levels, torch.from_numpy(make_batch(kind, B, n)).cuda())
    sha = z[f"{cfg}_{kind}_sha"]
    for lv, (p, c, _) in enumerate(out):
        rows = torch.cat((p, c), dim=2).cpu().numpy()
        for b in range(B):
            assert _sha_rows(rows[b]) == sha[b, lv].tobytes(), f"{cfg} {kind} cloud {b} level {levels[lv]}"
    assert not z[f"{cfg}_{kind}_glibc_extra"].any() and not z[f"{cfg}_{kind}_columns_extra"].any()


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("third", [False, True])
def test_two_plans_on_two_streams_are_admitted(graphs, third):
    """VERDICT r4 (next 1): two NdtPlans at the C2 shape (16 x 100k -> 1000,
    CU share 1: each k_front alone spans the chip) run on two user streams at
    once, with no pipeline guard -- eagerly, or as two HIP graphs replayed on
    the two streams.  No cloud barrier times out: every cloud has rc 0 and
    both batches equal the full-size fixture digests (the oracle's rows) after
    every round.  Two share-1 plans are within the bound of k_front's
    cloud-major deal (15 + 15 partial workgroups < 32 CUs per XCD), so their
    launches overlap unadmitted (include/ndnet_amd.h ndnet_ndt_set_path);
    with a third live share-1 plan (``third``) the front lanes admit them, and
    the two plans' k_front spans do not overlap."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    z = golden("fullsize_rows.npz")
    B, n = int(z["batch"]), int(z["points"])
    k = int(z["levels_C2"][0])
    plans, ins, outs, shas = [], [], [], []
    idle = NdtPlan(B, n, k, -1) if third else None  # live, never run: engages the admission
    for kind in ("U", "L"):
        pl = NdtPlan(B, n, k, -1)
        assert pl.path == 2 and pl.front_lanes[1] == 4  # share 1: the whole chip
        plans.append(pl)
        ins.append(torch.from_numpy(make_batch(kind, B, n)).cuda())
        outs.append(torch.zeros((B, k, 12), dtype=torch.float32, device="cuda"))
        shas.append(z[f"C2_{kind}_sha"])
    from ndnet import _lib
    for pl in plans:  # k_front's per-workgroup start / end stamps (s_memrealtime: one clock for the chip)
        assert _lib.lib().ndnet_ndt_set_timing(pl.handle, 2) == 0
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    if graphs:
        gs = []
        for i in range(2):  # warm-up run, then capture on the stream it replays on
            with torch.cuda.stream(streams[i]):
                plans[i].run(ins[i], None, outs[i], None)
        torch.cuda.synchronize()
        for i in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=streams[i]):
                plans[i].run(ins[i], None, outs[i], None)
            gs.append(g)
        torch.cuda.synchronize()
    for rnd in range(3):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        for _ in range(2):  # two back-to-back runs per stream, interleaved on the host
            for i in range(2):
                with torch.cuda.stream(streams[i]):
                    if graphs:
                        gs[i].replay()
                    else:
                        plans[i].run(ins[i], None, outs[i], None)
        torch.cuda.synchronize()
        span = []
        for i in range(2):
            assert [st.rc for st in plans[i].host_stats()] == [0] * B, (graphs, rnd, i)
            plans[i].raise_sync_failures()
            rows = outs[i].cpu().numpy()
            for b in range(B):
                assert _sha_rows(rows[b]) == shas[i][b, 0].tobytes(), (graphs, rnd, i, b)
            G = ctypes.c_int(0)
            m = np.zeros(B * 256 * 2, np.uint64)
            assert _lib.lib().ndnet_ndt_debug_front_wg_marks(plans[i].handle, m.ctypes.data, ctypes.byref(G)) == 0
            m = m[: B * G.value * 2].reshape(B, G.value, 2).astype(np.int64)
            span.append((int(m[..., 0].min()), int(m[..., 1].max())))
        # admitted (third plan live): the two plans' last k_front launches (each
        # at CU share 1: all four front lanes) ran one after the other
        (a0, a1), (b0, b1) = span
        if third:
            assert a1 <= b0 or b1 <= a0, (graphs, rnd, span)
    del idle


def test_front_lanes_follow_the_cu_share():
    """A plan's k_front occupies ceil(4 * workgroups / CUs) front lanes: all 4
    at CU share 1, 2 at share 2 (so two share-2 plans can run side by side on
    disjoint lanes), none on the one-launch-per-stage path."""
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    a, b = NdtPlan(16, 100_000, 1000, -1), NdtPlan(16, 100_000, 1000, -1)
    assert a.front_lanes[1] == 4 and b.front_lanes[1] == 4
    a.set_cu_share(2, 1)
    b.set_cu_share(2, 1)
    (a0, an), (b0, bn) = a.front_lanes, b.front_lanes
    assert an == bn == 2
    assert {a0 % 4, (a0 + 1) % 4}.isdisjoint({b0 % 4, (b0 + 1) % 4})
    b.set_path(1)
    assert b.front_lanes[1] == 0


def test_front_barrier_timeout_fails_clouds_cleanly():
    """VERDICT r1 (weak 8): the NDNET_ERR_SYNC path of k_front's cloud
    barriers.  With a 1-tick timeout, a workgroup that reaches a barrier before
    its siblings gives up at once and fails its cloud: such clouds report
    rc -22 and all-zero rows, the launch still completes, and with the default
    timeout restored the same plan (its barrier words re-armed by the last
    workgroup out) runs the batch bit-exactly again."""
    import torch
    import oracle as O
    from ndnet import _lib
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    B, n, k = 4, 50_000, 500
    pts = make_batch("U", B, n, seed0=31)
    plan = NdtPlan(B, n, k, -1)
    assert plan.path == 2
    t = torch.from_numpy(pts).cuda()
    out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
    assert _lib.lib().ndnet_ndt_debug_set_sync_timeout(plan.handle, 1) == 0
    plan.run(t, None, out, None)
    torch.cuda.synchronize()
    st = plan.host_stats()
    rcs = [s.rc for s in st]
    assert -22 in rcs and set(rcs) <= {0, -22}, rcs
    o = out.cpu().numpy()
    for b in range(B):
        if rcs[b] == -22:
            assert not o[b].any()
    assert _lib.lib().ndnet_ndt_debug_set_sync_timeout(plan.handle, 0) == 0
    # never silent: the timeout set a flag in host memory, and the plan's next
    # call raises it (no synchronisation, whatever `check` says) -- once
    from ndnet.preprocessing.ndtnet_preprocessing import NdtCloudError
    with pytest.raises(NdtCloudError, match="-22"):
        plan.run(t, None, out, None)
    plan.run(t, None, out, None)
    torch.cuda.synchronize()
    assert all(s.rc == 0 for s in plan.host_stats())
    o = out.cpu().numpy()
    for b in range(B):
        pc, cov, r = O.downsample_f32(pts[b], k)
        assert r.rc == 0 and np.array_equal(o[b, :, :3], pc) and np.array_equal(o[b, :, 3:], cov)


@pytest.mark.parametrize("k", [1300, 2000, 2400, 2600])
def test_merge_paths_match_oracle(k):
    """The three k_kl_merge forms by list size: k = 1000 runs the all-LDS merge
    (every other test), k = 1300, 2000 (C5's first level) and 2400 the
    score-runs-in-LDS form with k_kl_nan_keys (35-72 chunks), k = 2600 the
    global-memory form (> 72 chunks; its prune also takes the global-memory
    walk).  Rows, event counts and the level-1 list against the oracle, on
    clouds whose prune removes NDs."""
    import torch
    import oracle as O
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing, last_stats
    from ndnet.synthetic import make_batch
    pts = make_batch("L", 2, 60_000, seed0=40)
    p, c, _ = ndt_preprocessing(k, torch.from_numpy(pts).cuda())
    p, c = p.cpu().numpy(), c.cpu().numpy()
    stats = last_stats()
    for b in range(2):
        pc, cov, r = O.downsample_f32(pts[b], k)
        assert stats[b].rc == r.rc == 0
        assert stats[b].num_events == len(r.ord_div) and stats[b].num_out == r.nout
        assert np.array_equal(p[b], pc) and np.array_equal(c[b], cov)


@pytest.mark.parametrize("k", [1000, 2000, 2600])
def test_merge_grid_stride_equals_one_group_per_workgroup(k):
    """Round 6: a plan at CU share s runs k_kl_merge on ceil(groups / s)
    workgroups per cloud, each merging several chunk groups after one staging
    of the runs (merge_grid, csrc/ndt_kernels.hip).  All three merge forms (k =
    1000: runs and NaN keys in LDS; 2000: runs in LDS; 2600: global memory)
    at share 2 (two chunk groups per workgroup) against the share-1 plan (one workgroup per group): rows,
    stats and every dumped list entry identical, on L clouds whose prune
    removes NDs (the lists built eagerly)."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    B, n = 16, 60_000
    pts = torch.from_numpy(make_batch("L", B, n, seed0=70)).cuda()
    res = []
    from ndnet import _lib
    for share in (1, 2):
        plan = NdtPlan(B, n, k, -1)
        plan.set_lazy_list(False)
        # the merge at both shares (a plan with a share sorts k = 1000 lists on k_kl_sort by default)
        _lib.check(_lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, 0), "set_list_sort")
        if share > 1:
            plan.set_cu_share(share)
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        plan.run(pts, None, out, None)
        torch.cuda.synchronize()
        st = plan.host_stats()
        assert all(x.rc == 0 for x in st), (share, [x.rc for x in st])
        dumps = [_dump(plan, b, int(st[b].num_nds), int(st[b].num_events)) for b in range(B)]
        res.append((out.cpu().numpy(), [bytes(x) for x in st], dumps))
        del plan
    o0, s0, d0 = res[0]
    assert any(x.num_nds > k for x in st)
    for o, s_, d in res[1:]:
        assert np.array_equal(o, o0) and s_ == s0
        for b in range(B):
            for key in ("ord_val", "ord_p", "ord_q", "alive"):
                assert np.array_equal(d[b][key], d0[b][key], equal_nan=True), (b, key)


@pytest.mark.parametrize("case", ["L", "L_nofuse", "L_rank_sort", "L_rank_sort_nofuse", "U_levels", "labelled"])
def test_list_sort_equals_merge(case):
    """Round 6: a plan whose event list fits one workgroup's LDS (k <= 1065)
    sorts each cloud's list on one workgroup (k_kl_sort: the chunk runs merged
    pairwise, then the NaN run) instead of k_kl_merge's workgroups per chunk
    group.  Both orders are the composite (key, slot) order: rows, classes,
    stats and every dumped list entry identical -- eager lists on L clouds
    whose prune removes NDs (with the prune fused into the sort's workgroup,
    and on k_kl's own launch), with the chunks ranked by a launch of their
    own (the default) and in the sort's launch (form 3: k_kl_rank_sort), U
    clouds' deferred lists built on demand for two further prune levels, and
    a labelled batch."""
    import torch
    from ndnet import _lib
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    kind = "U" if case.startswith("U") else "L"
    B, n = 12, 60_000
    pts = torch.from_numpy(make_batch(kind, B, n, seed0=90)).cuda()
    k = 1000 if case == "U_levels" else 800
    ncls = 27 if case == "labelled" else -1
    lbl = None
    if case == "labelled":
        lbl = torch.from_numpy(np.random.default_rng(9).integers(0, ncls + 1, size=(B, n)).astype(np.int32)).cuda()
    res = []
    for sort in (1, 0):
        plan = NdtPlan(B, n, k, ncls)
        plan.set_lazy_list(case == "U_levels")
        form = 3 if sort and case.startswith("L_rank_sort") else sort
        _lib.check(_lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, form), "set_list_sort")
        assert _lib.lib().ndnet_ndt_debug_get_list_sort(plan.handle) == sort
        if case.endswith("nofuse"):
            _lib.check(_lib.lib().ndnet_ndt_debug_set_kl_fuse(plan.handle, 0), "set_kl_fuse")
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        oc = None if lbl is None else torch.empty((B, k, ncls + 1), dtype=torch.float32, device="cuda")
        plan.run(pts, lbl, out, oc)
        levels = []
        if case == "U_levels":
            for k2 in (700, 400):
                o2 = torch.empty((B, k2, 12), dtype=torch.float32, device="cuda")
                plan.prune(k2, o2)
                levels.append(o2.cpu().numpy())
        torch.cuda.synchronize()
        st = plan.host_stats()
        assert all(x.rc == 0 for x in st), (sort, [x.rc for x in st])
        dumps = [_dump(plan, b, int(st[b].num_nds), int(st[b].num_events)) for b in range(B)]
        res.append((out.cpu().numpy(), None if oc is None else oc.cpu().numpy(), [bytes(x) for x in st], dumps,
                    levels))
        del plan
    (o1, c1, s1, d1, l1), (o0, c0, s0, d0, l0) = res
    if case != "U_levels":
        assert any(x.num_nds > k for x in st)
    assert np.array_equal(o1, o0) and s1 == s0
    if c1 is not None:
        assert np.array_equal(c1, c0)
    for a, b_ in zip(l1, l0):
        assert np.array_equal(a, b_)
    for b in range(B):
        for key in d1[b]:
            assert np.array_equal(d1[b][key], d0[b][key], equal_nan=True), (b, key)


def test_list_sort_form_by_list_size_and_share():
    """k_kl_sort takes the plans whose two key/slot buffers fit its LDS
    (ecap = 6 * (1.2 k + 1) <= 7680 slots: k <= 1065); larger lists keep
    k_kl_merge (test_merge_paths_match_oracle covers those).  By default
    (form 2) only a plan with a CU share takes it."""
    from ndnet import _lib
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    get = lambda p: _lib.lib().ndnet_ndt_debug_get_list_sort(p.handle)  # noqa: E731
    for k, fits in ((500, 1), (1000, 1), (1065, 1), (1070, 0), (2000, 0)):
        plan = NdtPlan(16, 100_000, k, -1)
        assert get(plan) == 0, k                    # share 1: the merge
        plan.set_cu_share(2)
        assert get(plan) == fits, k                 # a pipeline's share: the sort where it fits
        _lib.check(_lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, 0), "set_list_sort")
        assert get(plan) == 0, k
        _lib.check(_lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, 1), "set_list_sort")
        assert get(plan) == fits, k
        del plan
    assert _lib.lib().ndnet_ndt_debug_set_list_sort(None, 1) != 0
    plan = NdtPlan(2, 20_000, 500, -1)
    assert _lib.lib().ndnet_ndt_debug_set_list_sort(plan.handle, 4) != 0


def test_front_staged_scatter_active_at_c2():
    """The staged scatter actually runs for the C2 shape at CU share 1
    (16 x 100k points -> 1000 NDs): round 3's u16 histograms had shrunk the
    plan's LDS below the records' need and turned it off silently."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    plan = NdtPlan(16, 100_000, 1000, -1, device=torch.device("cuda", 0))
    assert plan.path == 2 and plan.front_staged
    plan.set_front_staged(False)
    assert not plan.front_staged


@pytest.mark.parametrize("case", ["U", "L", "labelled"])
def test_front_staged_scatter_equals_direct(case):
    """k_front's staged scatter (points placed in ND order in LDS, stored as
    consecutive dwords) against the per-lane 12-byte stores: the grouped
    points feed the order-dependent Welford, so equal means / covariances /
    KL lists / rows / one-hot classes show the runs are identical."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    kind = "L" if case == "labelled" else case
    pts = make_batch(kind, 8, 60_000, seed0=31)
    B, n, _ = pts.shape
    k, ncls = 800, (27 if case == "labelled" else -1)
    lbl = None
    if case == "labelled":
        lbl = torch.from_numpy(np.random.default_rng(3).integers(0, ncls + 1, size=(B, n)).astype(np.int32)).cuda()
    res = {}
    for staged in (True, False):
        plan = NdtPlan(B, n, k, ncls)
        plan.set_front_staged(staged)
        assert plan.path == 2
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        oc = None if lbl is None else torch.empty((B, k, ncls + 1), dtype=torch.float32, device="cuda")
        plan.run(torch.from_numpy(pts).cuda(), lbl, out, oc)
        torch.cuda.synchronize()
        stats = plan.host_stats()
        dumps = [_dump(plan, b, int(stats[b].num_nds), int(stats[b].num_events)) for b in range(B)]
        res[staged] = (out.cpu().numpy(), None if oc is None else oc.cpu().numpy(), stats, dumps)
    (o1, c1, s1, d1), (o0, c0, s0, d0) = res[True], res[False]
    assert np.array_equal(o1, o0)
    if c1 is not None:
        assert np.array_equal(c1, c0)
    for b in range(B):
        assert s1[b].rc == 0
        assert bytes(s1[b]) == bytes(s0[b]), f"cloud {b} stats"
        for key in d1[b]:
            assert np.array_equal(d1[b][key], d0[b][key], equal_nan=True), (b, key)


@pytest.mark.parametrize("case", ["U", "L", "labelled", "L1300", "C5"])
def test_fused_prune_equals_k_kl(case):
    """The prune + rows on the merge launch's last workgroup per cloud (the
    default) against k_kl's own launch: rows, classes, stats and every dumped
    intermediate (the built list, alive flags, post-KL covariances) equal.
    k = 1000 fuses into the all-LDS merge, k = 1300 into the score-runs-in-LDS
    merge; C5 runs two further prune levels off the fused level-1 list."""
    import torch
    from ndnet import _lib
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    kind = "U" if case == "U" else "L"
    pts = make_batch(kind, 6, 60_000, seed0=47)
    B, n, _ = pts.shape
    k = 1300 if case == "L1300" else (1000 if case == "C5" else 800)
    ncls = 27 if case == "labelled" else -1
    lbl = None
    if case == "labelled":
        lbl = torch.from_numpy(np.random.default_rng(5).integers(0, ncls + 1, size=(B, n)).astype(np.int32)).cuda()
    res = {}
    for fuse in (1, 0):
        plan = NdtPlan(B, n, k, ncls)
        plan.set_lazy_list(case == "U")  # U: the deferred lists through the fused launch too
        _lib.check(_lib.lib().ndnet_ndt_debug_set_kl_fuse(plan.handle, fuse), "set_kl_fuse")
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        oc = None if lbl is None else torch.empty((B, k, ncls + 1), dtype=torch.float32, device="cuda")
        plan.run(torch.from_numpy(pts).cuda(), lbl, out, oc)
        levels = []
        if case == "C5":
            for k2 in (700, 400):
                o2 = torch.empty((B, k2, 12), dtype=torch.float32, device="cuda")
                plan.prune(k2, o2)
                levels.append(o2.cpu().numpy())
        torch.cuda.synchronize()
        stats = plan.host_stats()
        dumps = [_dump(plan, b, int(stats[b].num_nds), int(stats[b].num_events)) for b in range(B)]
        res[fuse] = (out.cpu().numpy(), None if oc is None else oc.cpu().numpy(), stats, dumps, levels)
    (o1, c1, s1, d1, l1), (o0, c0, s0, d0, l0) = res[1], res[0]
    assert np.array_equal(o1, o0)
    if c1 is not None:
        assert np.array_equal(c1, c0)
    for a, b_ in zip(l1, l0):
        assert np.array_equal(a, b_)
    for b in range(B):
        assert s1[b].rc == 0
        assert bytes(s1[b]) == bytes(s0[b]), f"cloud {b} stats"
        for key in d1[b]:
            assert np.array_equal(d1[b][key], d0[b][key], equal_nan=True), (b, key)


def test_run_parts_equal_whole_run():
    """ndnet_ndt_set_run_part: the front (part 1) and the rest (part 2) as two
    stream-ordered calls give the rows and stats of one whole run."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    pts = torch.from_numpy(make_batch("L", 4, 40_000, seed0=41)).cuda()
    res = []
    for parts in ((0,), (1, 2)):
        plan = NdtPlan(4, 40_000, 500, -1)
        out = torch.empty((4, 500, 12), dtype=torch.float32, device="cuda")
        for part in parts:
            plan.run(pts, None, out, None, part=part)
        torch.cuda.synchronize()
        res.append((out.cpu().numpy(), [bytes(s) for s in plan.host_stats()]))
    assert np.array_equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]


@pytest.mark.parametrize("num_classes", [28, 300, 3])
def test_full_size_labelled(num_classes):
    """SURVEY 8(f)2 at the bench's size: 16 x 100k labelled L clouds -> 1000
    NDs, every cloud's rows and one-hot classes against the oracle
    (normal_distributions.c:107-121 first-max argmax; ndtnet_preprocessing.py:
    22,55-57 one-hot).  28 classes: the training config, labels from
    make_labelled_batch, through ndt_preprocessing's one-hot argmax (the
    reference driver's path, ndtnet_preprocessing.py:34).  300 classes: 301
    bins x 64 NDs per k_welford_q workgroup exceed the LDS histogram budget
    (kWqHistMax, 64 KB), so the per-ND histograms live in global memory; labels
    uniform over all 301 values, so the first-max tie rule decides many NDs.
    3 classes, uniform labels: the LDS histograms the whole quad adds into,
    with near-ties in every ND (4 bins, ~100 labels each)."""
    import torch
    import oracle as O
    from ndnet.preprocessing.ndtnet_preprocessing import ndt_preprocessing, last_stats
    from ndnet.synthetic import make_labelled_batch
    B, n, k = 16, 100_000, 1000
    if num_classes == 28:
        pts, onehot = make_labelled_batch(B, n, num_classes, seed0=0)
        labels = onehot.argmax(axis=2)
        p, c, g = ndt_preprocessing(k, torch.from_numpy(pts).cuda(), torch.from_numpy(onehot).cuda(), num_classes)
        p, c, g = p.cpu().numpy(), c.cpu().numpy(), g.cpu().numpy()
        stats = last_stats()
    else:
        pts, _ = make_labelled_batch(B, n, 1, seed0=0)
        labels = np.random.default_rng(5).integers(0, num_classes + 1, (B, n))
        plan, out, g = _run_plan(pts, k, labels, num_classes, exact_counts=False)
        p, c = out[..., :3], out[..., 3:]
        stats = plan.host_stats()
    assert g.shape == (B, k, num_classes + 1)
    for b in range(B):
        r = O.run(pts[b].astype(np.float64), k, classes=labels[b], num_classes=num_classes)
        assert stats[b].rc == r.rc == 0
        rows = _f32_rows(r.out_pc, r.out_cov, k)
        assert np.array_equal(p[b], rows[:, :3]), f"cloud {b} means"
        assert np.array_equal(c[b], rows[:, 3:]), f"cloud {b} covariances"
        onehot_ref = np.zeros((k, num_classes + 1), np.float32)
        onehot_ref[np.arange(k), r.out_cls] = 1.0
        assert np.array_equal(g[b], onehot_ref), f"cloud {b} classes"
    if num_classes == 300:  # the tie rule and the wide histogram are exercised
        assert len(np.unique(g.argmax(axis=2))) > 100
    if num_classes == 3:
        assert len(np.unique(g.argmax(axis=2))) == 4


@pytest.mark.parametrize("share,k", [(2, 1000), (2, 2000)])
def test_cu_share_results_identical(share, k):
    """ndnet_ndt_set_cu_share: k_front on CUs / (share B) workgroups per cloud
    and k_welford_q on CUs / share give the same rows and stats, bit for bit,
    as the whole-chip plan (U and L clouds, 16 x 100k -> 1000 (C2) and -> 2000
    (C5's first level: 13 bins per workgroup, which fit since the rank-bin
    histograms are u16)).  A share whose k_front does not fit (4: 25 bins per
    workgroup exceed its LDS) is refused and the plan keeps its previous share."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    B, n = 16, 100_000
    for kind in ("U", "L"):
        pts = torch.from_numpy(make_batch(kind, B, n)).cuda()
        res = []
        for s in (1, share):
            plan = NdtPlan(B, n, k, -1)
            assert plan.path == 2
            if s > 1:
                plan.set_cu_share(s)
                with pytest.raises(RuntimeError):
                    plan.set_cu_share(4)
            out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
            plan.run(pts, None, out, None)
            torch.cuda.synchronize()
            res.append((out.cpu().numpy(), [bytes(st) for st in plan.host_stats()]))
        assert np.array_equal(res[0][0], res[1][0]) and res[0][1] == res[1][1], kind


def _run_thresholds(pts, k, thresholds, path=2, labels=None, num_classes=-1, forms=("auto",)):
    """One plan per heavy threshold (and k_welford_q light form) over the
    same batch: rows, one-hot classes, stats and every dumped intermediate
    (counts, means, pre- and post-KL covariances, list, kept set)."""
    import torch
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    B, n, _ = pts.shape
    res = []
    for t, form in ((t, f) for t in thresholds for f in forms):
        plan = NdtPlan(B, n, k, num_classes)
        plan.set_path(path)
        plan.set_lazy_list(False)
        plan.set_heavy_threshold(t)
        plan.set_welford_form(form)
        out = torch.empty((B, k, 12), dtype=torch.float32, device="cuda")
        lbl = None if labels is None else torch.from_numpy(labels.astype(np.int32)).cuda()
        oc = None if labels is None else torch.empty((B, k, num_classes + 1), dtype=torch.float32, device="cuda")
        plan.run(torch.from_numpy(np.ascontiguousarray(pts, dtype=np.float32)).cuda(), lbl, out, oc)
        torch.cuda.synchronize()
        stats = plan.host_stats()
        dumps = [_dump(plan, b, int(stats[b].num_nds), int(stats[b].num_events)) if stats[b].rc == 0 else None
                 for b in range(B)]
        res.append((out.cpu().numpy(), None if oc is None else oc.cpu().numpy(),
                    [bytes(st) for st in stats], dumps, [int(st.num_nds) for st in stats]))
    return res


def _same(res):
    o0, c0, s0, d0, _ = res[0]
    for o, c, s, d, _ in res[1:]:
        assert np.array_equal(o, o0)
        assert (c is None and c0 is None) or np.array_equal(c, c0)
        assert s == s0
        for b in range(len(d0)):
            if d0[b] is None:
                assert d[b] is None
                continue
            for key in d0[b]:
                assert np.array_equal(d[b][key], d0[b][key], equal_nan=True), (b, key)


@pytest.mark.parametrize("path", [1, 2])
def test_heavy_nds_equal_quad_path(path):
    """k_welford_q's whole-wave path for long NDs (wq_heavy: the mean
    recurrence on three lanes, per-sample products on 64, ordered sums on
    six) against the lane-quad path: threshold 1 (every ND on a wave), 256
    (the default), 2^31 (none), on clouds of few NDs (4096..20000 points -> 8..40
    NDs: 100..2500 samples per ND, partial last blocks of every length) and
    L clouds, with both binning paths; bit for bit, and the rows equal the
    oracle's."""
    import oracle as O
    from ndnet.synthetic import make_batch
    rng = np.random.default_rng(11)
    few = np.stack([rng.uniform(-5, 5, (20_000, 3)).astype(np.float32),
                    make_batch("L", 1, 20_000, seed0=3)[0],
                    np.concatenate([rng.normal(0, 0.3, (12_000, 3)), rng.uniform(-9, 9, (8_000, 3))]).astype(np.float32)])
    for pts, k in ((few, 8), (few, 40), (make_batch("L", 4, 50_000, seed0=40), 500)):
        res = _run_thresholds(pts, k, (1, 256, 1 << 31), path=path)
        _same(res)
        for b in range(len(pts)):
            pc, cov, r = O.downsample_f32(pts[b], k)
            assert res[0][2][b] is not None
            if r.rc == 0:
                assert np.array_equal(res[0][0][b, :, :3], pc) and np.array_equal(res[0][0][b, :, 3:], cov), b
        if k == 8:  # heavy NDs present at the default threshold
            assert any(d is not None and d["nd_n"].max() >= 256 for d in res[0][3])


def test_heavy_nds_labelled_and_full_size():
    """The labelled path (class histograms of heavy NDs on their own wave) and
    the full-size L batch (16 x 100k -> 1000: the default threshold's heavy
    NDs, up to 1675 samples) equal the all-quad path bit for bit."""
    from ndnet.synthetic import make_batch
    rng = np.random.default_rng(12)
    pts = make_batch("L", 3, 20_000, seed0=8)
    lbl = rng.integers(0, 29, (3, 20_000))
    _same(_run_thresholds(pts, 30, (1, 256, 1 << 31), labels=lbl, num_classes=28))
    _same(_run_thresholds(make_batch("L", 16, 100_000), 1000, (256, 1 << 31)))


@pytest.mark.parametrize("labelled", [False, True])
def test_welford_forms_equal(labelled):
    """k_welford_q's two light forms (light64: one ND per lane; quad: a lane
    quad per ND -- a plan picks by its CU share, include/ndnet_amd.h
    ndnet_ndt_set_welford_form) with the heavy threshold at 256 and at 2^31
    (every ND light): identical rows, classes, stats and intermediates, on U
    and L clouds at full size and on a labelled L batch; the default form is
    quad at CU share 1 and light64 at share 2."""
    from ndnet.preprocessing.ndtnet_preprocessing import NdtPlan
    from ndnet.synthetic import make_batch
    if labelled:
        rng = np.random.default_rng(13)
        pts = make_batch("L", 3, 20_000, seed0=9)
        lbl = rng.integers(0, 29, (3, 20_000))
        _same(_run_thresholds(pts, 30, (256, 1 << 31), labels=lbl, num_classes=28, forms=("light64", "quad")))
        return
    for kind in ("U", "L"):
        _same(_run_thresholds(make_batch(kind, 16, 100_000), 1000, (256, 1 << 31), forms=("light64", "quad")))
    plan = NdtPlan(16, 100_000, 1000, -1)
    assert plan.welford_form == "quad"
    plan.set_cu_share(2)
    assert plan.welford_form == "light64"
    plan.set_welford_form("quad")
    assert plan.welford_form == "quad"


def test_heavy_nds_float64_and_out_of_range():
    """Double input (the legacy ABI's ndnet_ndt_run_f64) with heavy NDs: a
    plain cloud, and one with coordinates outside the fast path's range
    (|x| = 1e-95 < 2^-300: the wave refolds those NDs with IEEE divisions),
    against the oracle's legacy chain."""
    import oracle as O
    from ndnet.preprocessing.ndt_legacy import NDT_Sampler
    rng = np.random.default_rng(13)
    for tiny in (False, True):
        a = rng.uniform(-5, 5, (6000, 3))
        if tiny:
            a[::7, 1] = 1e-95 * np.sign(a[::7, 1])
        s = NDT_Sampler(a)
        pc, cov, _ = s.downsample(16)
        ref = O.LegacyChain(a)
        pc2, cov2 = ref.downsample(16)
        assert np.array_equal(pc, pc2, equal_nan=True) and np.array_equal(cov, cov2, equal_nan=True), tiny
        s.cleanup()
        ref.cleanup()


def _lu_cases(seed):
    """3x3 matrices for the LU chain: random covariances (SPD and rank-1),
    random general matrices, ties between pivot candidates, zero / negative-zero
    columns, pivots below DBL_MIN, huge and tiny entries, NaN and inf."""
    rng = np.random.default_rng(seed)
    mats = []
    for _ in range(2000):
        a = rng.normal(size=(3, 3))
        mats.append(a @ a.T)
    for _ in range(500):
        v = rng.normal(size=3)
        mats.append(np.outer(v, v))
    mats += list(rng.normal(size=(1500, 3, 3)))
    mats += list(rng.integers(-2, 3, size=(1500, 3, 3)).astype(np.float64))  # ties and exact zeros
    for _ in range(300):
        a = rng.normal(size=(3, 3))
        a[:, rng.integers(0, 3)] = 0.0
        a[rng.integers(0, 3), rng.integers(0, 3)] = -0.0
        mats.append(a)
    for scale in (1e-310, 1e-300, 1e300, 3e307):
        mats += list(rng.normal(size=(100, 3, 3)) * scale)
    a = rng.normal(size=(50, 3, 3))
    a[:, 0, 0] = np.nan
    mats += list(a)
    a = rng.normal(size=(50, 3, 3))
    a[:, 1, 2] = np.inf
    mats += list(a)
    return np.ascontiguousarray(np.array(mats, dtype=np.float64).reshape(-1, 9))


def test_lu_chain_matches_oracle():
    """The device LU chain (lu3 + event flags, run by k_welford_q's group
    hand-off for every ND) against the oracle's GSL 2.7.1 LU_decomp
    restatement: every state, permutation, sign and flag of 12 chained
    decompositions, bit for bit, on ~6000 matrices with ties, zeros,
    sub-DBL_MIN pivots, huge / tiny entries, NaN and inf."""
    import torch
    import oracle as O
    from ndnet import _lib
    A = _lu_cases(21)
    n, steps = len(A), 12
    st_h = np.zeros((n, steps, 9))
    ps_h = np.zeros((n, steps), np.uint32)
    fl_h = np.zeros((n, steps), np.uint32)
    O.lib().orc_lu_chain(O._ptr(A), ctypes.c_uint64(n), ctypes.c_int(steps), O._ptr(st_h), O._ptr(ps_h),
                         O._ptr(fl_h))
    dA = torch.from_numpy(A).cuda()
    st = torch.empty((n, steps, 9), dtype=torch.float64, device="cuda")
    ps = torch.empty((n, steps), dtype=torch.int32, device="cuda")
    fl = torch.empty((n, steps), dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib().ndnet_debug_lu_chain(dA.data_ptr(), n, steps, st.data_ptr(), ps.data_ptr(), fl.data_ptr(),
                                               torch.cuda.current_stream().cuda_stream), "debug_lu_chain")
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    nan = np.isnan(st_h)  # NaN payloads may differ; every other value bit for bit (signed zeros too)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got.view(np.uint64)[~nan], st_h.view(np.uint64)[~nan])
    assert np.array_equal(ps.cpu().numpy().astype(np.uint32), ps_h)
    assert np.array_equal(fl.cpu().numpy().astype(np.uint32), fl_h)
