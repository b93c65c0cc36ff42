"""The reference-structured CPU baseline (oracle/cpu_ref.c, what bench.py's
cpu_baseline times) computes what the oracle computes: its structure (8
pthreads, a mutex per voxel, heap traffic per KL call, -O0) changes the run
time, not the result -- up to the thread interleaving of the Welford updates,
which the reference's 8-thread build has too."""
import numpy as np

import oracle as O


def test_cpu_ref_matches_oracle():
    """C2-U (100k -> 1000: all 1000 voxels of the 10^3 grid kept, the prune
    removes none): the same rows; means to rounding (their summation order
    follows the threads).  Where the prune removes NDs the kept set is
    chaotic in that order, so only the return code and the row
    count are compared there."""
    from ndnet.synthetic import uniform_cloud, lidar_cloud
    pts = uniform_cloud(100_000, 0).astype(np.float64)
    r = O.run(pts, 1000)
    pc, cov, rc = O.cref_downsample(pts, 1000)
    assert rc == r.rc == 0 and r.search.num_nds == 1000
    assert np.allclose(pc, r.out_pc, rtol=0, atol=1e-12)
    for pts32, k in ((lidar_cloud(20_000, 2), 300), (uniform_cloud(4096, 0), 256)):
        pts = pts32.astype(np.float64)
        r = O.run(pts, k)
        pc, cov, rc = O.cref_downsample(pts, k)
        assert rc == r.rc == 0
        assert (np.abs(pc).sum(1) > 0).sum() == (np.abs(r.out_pc).sum(1) > 0).sum() == k


def test_cpu_ref_estimate_counts():
    from ndnet.synthetic import lidar_cloud
    pts = lidar_cloud(30_000, 4).astype(np.float64)
    r = O.run(pts, 500)
    s = r.search
    assert O.cref_estimate_only(pts, s.voxel_size, s.len, s.off) == s.num_nds


def test_cpu_ref_failure_code():
    rng = np.random.default_rng(5)
    flat = rng.uniform(-5, 5, (4101, 3))
    flat[:, 2] = 1.5
    _, _, rc = O.cref_downsample(flat, 200)
    assert rc == O.run(flat, 200).rc == -3
