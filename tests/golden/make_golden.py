#!/usr/bin/env python3
"""Generate the committed parity fixtures under tests/golden/ (build container only).

Sources, in order of authority:
  * the reference's own estimate stage -- core_legacy/src/{normal_distributions,
    voxel,pointclouds,matrix}.c compiled unmodified into oracle/_ref -- for the
    bisection (guesses, counts, grid) and the per-voxel counts, means, pre-KL
    covariances and classes (bit-exact);
  * the reference's own Python model (ndnet/models/ndtnet.py, imported from
    /root/reference under the name ``refndnet``) for NDTNetSegmentation outputs;
  * the reference's own ctypes driver (ndt_legacy.py / ndtnet_preprocessing.py)
    run against the CPU oracle's legacy ABI, for the end-to-end float32 rows;
  * the CPU oracle (oracle/ndt_oracle.c) for the KL list, its order, the kept
    set and the emitted rows -- "parity unpinned" against GSL (absent here).
Nothing from /root/reference is copied: fixtures hold inputs and outputs only.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes
import importlib
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
sys.path.insert(0, HERE)

import oracle as O  # noqa: E402
from ndnet.synthetic import lidar_cloud, uniform_cloud  # noqa: E402
from model_init import deterministic_state  # noqa: E402

REF_ROOT = "/root/reference"


def load_reference(lib_redirect: str | None = None):
    """Import the reference ``ndnet`` package as ``refndnet``; its hard-coded
    /usr/local/lib/libndnet.so load is redirected (to ``lib_redirect`` or to an
    inert stand-in when only the torch model is needed)."""
    for k in [k for k in sys.modules if k == "refndnet" or k.startswith("refndnet.")]:
        del sys.modules[k]
    spec = importlib.util.spec_from_file_location("refndnet", f"{REF_ROOT}/ndnet/__init__.py",
                                                  submodule_search_locations=[f"{REF_ROOT}/ndnet"])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["refndnet"] = mod
    spec.loader.exec_module(mod)
    real = ctypes.cdll.LoadLibrary

    class _Inert:
        def __getattr__(self, k):
            return types.SimpleNamespace(argtypes=None)

    def fake(path):
        if "libndnet" in str(path):
            return real(lib_redirect) if lib_redirect else _Inert()
        return real(path)

    ctypes.cdll.LoadLibrary = fake
    try:
        model = importlib.import_module("refndnet.models.ndtnet")
        pre = importlib.import_module("refndnet.preprocessing.ndtnet_preprocessing")
    finally:
        ctypes.cdll.LoadLibrary = real
    return model, pre


CLOUDS = [("U", 4096, 256, 0), ("U", 4096, 256, 1), ("L", 4096, 256, 0), ("L", 4096, 256, 1),
          ("U", 2003, 128, 7)]  # n % 8 = 3: the dropped tail


def ndt_fixtures() -> None:
    assert O.ref_lib() is not None, "oracle/_ref not built (make -C oracle)"
    for kind, n, k, seed in CLOUDS:
        gen = uniform_cloud if kind == "U" else lidar_cloud
        pts32 = gen(n, seed)
        pts = pts32.astype(np.float64)
        # reference estimate stage: bisection + per-voxel state at the accepted size
        rc, guesses, counts, ln, off, vs = O.ref_search(pts, k)
        assert rc == 0
        cnt, mean, cov, _, nn = O.ref_estimate(pts, vs, ln, off)
        # labelled variant (class histogram argmax, normal_distributions.c:107-121)
        rng = np.random.default_rng(100 + seed)
        ncls = 5
        labels = rng.integers(0, ncls + 1, n).astype(np.uint16)
        _, _, _, cls, _ = O.ref_estimate(pts, vs, ln, off, classes=labels, num_classes=ncls)
        # the oracle's full path (KL / order / prune / rows), portable log
        r = O.run(pts, k, classes=labels, num_classes=ncls, portable_log=True)
        assert r.rc == 0
        assert np.array_equal(r.vox_n, cnt) and np.array_equal(r.vox_mean, mean) and np.array_equal(r.vox_cov_pre, cov)
        assert np.array_equal(r.vox_cls[cnt > 0], cls[cnt > 0])
        rl = O.run(pts, k, portable_log=False)  # glibc log
        name = f"ndt_{kind}{n}_k{k}_s{seed}.npz"
        np.savez_compressed(
            os.path.join(HERE, name),
            points=pts32, k=k, labels=labels, num_classes=ncls,
            ref_guesses=guesses, ref_counts=counts, ref_len=np.array(ln), ref_off=off, ref_voxel_size=vs,
            ref_count=cnt, ref_mean=mean, ref_cov=cov, ref_cls=cls,
            orc_ev_div=r.ev_div, orc_ev_p=r.ev_p, orc_ev_q=r.ev_q, orc_ev_rc=r.ev_rc,
            orc_ord_div=r.ord_div, orc_ord_p=r.ord_p, orc_ord_q=r.ord_q,
            orc_post_div=r.post_div, orc_post_p=r.post_p, orc_post_q=r.post_q, orc_post_nkl=r.post_nkl,
            orc_cov_post=r.vox_cov_post, orc_kept=r.vox_kept, orc_prune_rc=r.prune_rc, orc_num_valid=r.num_valid,
            orc_out_pc=r.out_pc, orc_out_cov=r.out_cov, orc_out_cls=r.out_cls, orc_nout=r.nout,
            orc_glibc_kept=rl.vox_kept, orc_glibc_out_cov=rl.out_cov)
        print("wrote", name, "V", len(cnt), "valid", int((cnt > 0).sum()), "events", len(r.ev_div))


def preprocessing_fixture() -> None:
    """The reference's batch driver, unchanged, over the oracle's legacy ABI."""
    import torch
    _, pre = load_reference(lib_redirect=O.LIB)
    O.set_portable_log(True)
    B, n, k = 3, 4096, 256
    pts = np.stack([uniform_cloud(n, 20), lidar_cloud(n, 21), uniform_cloud(n, 22)])
    p, c, cl = pre.ndt_preprocessing(k, torch.from_numpy(pts))
    np.savez_compressed(os.path.join(HERE, "preproc_B3_k256.npz"), points=pts, k=k, out_points=p.numpy(),
                        out_covs=c.numpy())
    print("wrote preproc_B3_k256.npz")


def model_fixture() -> None:
    import torch
    model_mod, _ = load_reference()
    torch.manual_seed(0)
    for F, C, B, N in [(768, 28, 2, 64), (64, 5, 2, 40)]:
        m = model_mod.NDTNetSegmentation(3, C, F)
        m.load_state_dict(deterministic_state(m.state_dict()))
        rng = np.random.default_rng(F + C)
        pts = rng.uniform(-10, 10, (B, N, 3)).astype(np.float32)
        covs = rng.normal(0, 1, (B, N, 9)).astype(np.float32)
        with torch.no_grad():
            m.eval()
            out_eval = m(torch.from_numpy(pts), torch.from_numpy(covs)).numpy()
            m.train()
            out_train = m(torch.from_numpy(pts), torch.from_numpy(covs)).numpy()
        name = f"ndtnet_seg_F{F}_C{C}.npz"
        np.savez_compressed(os.path.join(HERE, name), points=pts, covs=covs, feature_dim=F, num_classes=C,
                            out_eval=out_eval, out_train=out_train)
        print("wrote", name)


def model_train_fixture() -> None:
    """A well-conditioned train-mode fixture: 16 clouds, each at its own scale
    and offset, so the TNet FC heads' BatchNorm1d (batch statistics over the
    clouds) divides by the features' real spread, not by ~sqrt(eps) as with
    the 2-cloud fixtures above.  out_train: the reference module's fp32 train
    forward; out_train64: the same module in float64."""
    import copy
    import torch
    model_mod, _ = load_reference()
    F, C, B, N = 768, 28, 16, 128
    m = model_mod.NDTNetSegmentation(3, C, F)
    m.load_state_dict(deterministic_state(m.state_dict()))
    rng = np.random.default_rng(2024)
    scale = (0.5 + 0.25 * np.arange(B)).reshape(B, 1, 1)
    shift = rng.uniform(-5, 5, (B, 1, 3))
    pts = (rng.uniform(-10, 10, (B, N, 3)) * scale + shift).astype(np.float32)
    covs = (rng.normal(0, 1, (B, N, 9)) * scale).astype(np.float32)
    m64 = copy.deepcopy(m).double()
    with torch.no_grad():
        m.train()
        out_train = m(torch.from_numpy(pts), torch.from_numpy(covs)).numpy()
        m64.train()
        out64 = m64(torch.from_numpy(pts).double(), torch.from_numpy(covs).double()).numpy()
    name = f"ndtnet_seg_train_F{F}_C{C}_B{B}.npz"
    np.savez_compressed(os.path.join(HERE, name), points=pts, covs=covs, feature_dim=F, num_classes=C,
                        out_train=out_train, out_train64=out64)
    print("wrote", name, "fp32 vs float64:", float(np.abs(out_train - out64).max()))


if __name__ == "__main__":
    ndt_fixtures()
    preprocessing_fixture()
    model_fixture()
    model_train_fixture()
