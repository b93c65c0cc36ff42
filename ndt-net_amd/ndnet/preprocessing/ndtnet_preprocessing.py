"""Batched NDT preprocessing on the GPU.

Drop-in for ``ndnet.preprocessing.ndtnet_preprocessing.ndt_preprocessing``
(reference ndnet/preprocessing/ndtnet_preprocessing.py:6-73).  The reference
loops over the batch on the host, copies each cloud to the CPU as float64,
runs the C core and copies the result back; here the whole batch stays in HBM
and one call of ``ndnet_ndt_run`` (include/ndnet_amd.h) processes every cloud.
Results are bit-identical to the reference core's single-worker schedule
(SURVEY §8c), cast to float32 and passed through ``nan_to_num`` as the
reference does (ndtnet_preprocessing.py:66-69).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch

from .. import _lib


class NdtPlan:
    """Device workspace for one (batch, points, NDs, classes) shape."""

    def __init__(self, batch: int, num_points: int, num_nds: int, num_classes: int = -1,
                 voxel_capacity: int = 0, device: torch.device | None = None):
        _lib.require_gpu()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.batch, self.num_points, self.num_nds, self.num_classes = batch, num_points, num_nds, num_classes
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = _lib.lib().ndnet_ndt_plan_create(batch, num_points, num_nds, num_classes, voxel_capacity,
                                                  ctypes.byref(h))
        _lib.check(rc, "ndnet_ndt_plan_create")
        self.handle = h
        self.stats = torch.zeros((batch, _lib.STATS_BYTES), dtype=torch.uint8, device=self.device)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                with torch.cuda.device(self.device):
                    _lib.lib().ndnet_ndt_plan_destroy(h)
            except Exception:
                pass
            self.handle = None

    def run(self, points: torch.Tensor, labels: Optional[torch.Tensor], out: torch.Tensor,
            out_classes: Optional[torch.Tensor], part: int = 0) -> None:
        """part: 0 the whole run; 1 the front only (k_front); 2 the rest, after a
        part-1 call with the same arguments in stream order
        (include/ndnet_amd.h ndnet_ndt_set_run_part)."""
        assert points.is_contiguous() and points.dtype == torch.float32 and points.device == self.device
        assert out.is_contiguous() and out.shape == (self.batch, self.num_nds, 12)
        self.raise_sync_failures()
        st = _lib.stream_ptr(self.device)
        _lib.check(_lib.lib().ndnet_ndt_set_run_part(self.handle, int(part)), "ndnet_ndt_set_run_part")
        rc = _lib.lib().ndnet_ndt_run(
            self.handle, st, points.data_ptr(),
            labels.data_ptr() if labels is not None else None,
            out.data_ptr(),
            out_classes.data_ptr() if out_classes is not None else None,
            self.stats.data_ptr())
        if part:
            _lib.lib().ndnet_ndt_set_run_part(self.handle, 0)
        _lib.check(rc, "ndnet_ndt_run")

    def set_path(self, path: int) -> None:
        """1: one launch per stage; 2: the fused front kernel (k_front); 0: 2 where allowed."""
        _lib.check(_lib.lib().ndnet_ndt_set_path(self.handle, int(path)), "ndnet_ndt_set_path")

    def set_cu_share(self, front_share: int, welford_share: Optional[int] = None) -> None:
        """k_front on CUs / front_share, k_welford_q on CUs / welford_share
        (default: front_share) -- include/ndnet_amd.h ndnet_ndt_set_cu_share:
        leaves CUs to another stream; identical results."""
        ws = front_share if welford_share is None else welford_share
        _lib.check(_lib.lib().ndnet_ndt_set_cu_share(self.handle, int(front_share), int(ws)), "ndnet_ndt_set_cu_share")

    def set_exact_counts(self, on: bool) -> None:
        """Count every bisection grid, also those with fewer voxels than k
        (include/ndnet_amd.h ndnet_ndt_set_exact_counts; debug / parity)."""
        _lib.check(_lib.lib().ndnet_ndt_set_exact_counts(self.handle, 1 if on else 0), "ndnet_ndt_set_exact_counts")

    def set_front_staged(self, on: bool) -> None:
        """k_front's scatter through LDS records in ND order (default on;
        include/ndnet_amd.h ndnet_ndt_set_front_staged; identical results)."""
        _lib.check(_lib.lib().ndnet_ndt_set_front_staged(self.handle, 1 if on else 0), "ndnet_ndt_set_front_staged")

    @property
    def front_staged(self) -> bool:
        """Whether k_front's scatter runs staged for this plan's shapes (float input)."""
        rc = _lib.lib().ndnet_ndt_get_front_staged(self.handle)
        if rc < 0:
            _lib.check(rc, "ndnet_ndt_get_front_staged")
        return rc == 1

    def set_lazy_list(self, on: bool) -> None:
        """Defer the retained KL list of clouds whose level-1 prune cannot read
        it (num_nds <= k) until a prune or dump needs it (default on;
        include/ndnet_amd.h ndnet_ndt_set_lazy_list)."""
        _lib.check(_lib.lib().ndnet_ndt_set_lazy_list(self.handle, 1 if on else 0), "ndnet_ndt_set_lazy_list")

    def set_welford_form(self, form: str) -> None:
        """k_welford_q's light form: "light64" (one ND per lane), "quad" (a lane
        quad per ND) or "auto" (quad at CU share 1, light64 above: the default);
        identical results (include/ndnet_amd.h ndnet_ndt_set_welford_form)."""
        code = {"auto": 0, "light64": 1, "quad": 2}[form]
        _lib.check(_lib.lib().ndnet_ndt_set_welford_form(self.handle, code), "ndnet_ndt_set_welford_form")

    @property
    def welford_form(self) -> str:
        return {1: "light64", 2: "quad"}[_lib.lib().ndnet_ndt_get_welford_form(self.handle)]

    def set_heavy_threshold(self, min_samples: int) -> None:
        """NDs with at least ``min_samples`` points get a whole wave in
        k_welford_q (include/ndnet_amd.h ndnet_ndt_set_heavy_threshold;
        identical results, default 256)."""
        _lib.check(_lib.lib().ndnet_ndt_set_heavy_threshold(self.handle, int(min_samples)),
                   "ndnet_ndt_set_heavy_threshold")

    @property
    def path(self) -> int:
        return int(_lib.lib().ndnet_ndt_get_path(self.handle))

    @property
    def front_lanes(self) -> Tuple[int, int]:
        """(first lane, lane count) of the device's front lanes this plan's
        k_front occupies (include/ndnet_amd.h ndnet_ndt_get_front_lanes;
        count 0 on the one-launch-per-stage path)."""
        l0, nl = ctypes.c_int(0), ctypes.c_int(0)
        _lib.check(_lib.lib().ndnet_ndt_get_front_lanes(self.handle, ctypes.byref(l0), ctypes.byref(nl)),
                   "ndnet_ndt_get_front_lanes")
        return l0.value, nl.value

    def raise_sync_failures(self) -> None:
        """Raises ``NdtCloudError`` (rc -22) if a k_front cloud barrier of an
        earlier run of this plan timed out -- read from mapped host memory,
        without synchronising (include/ndnet_amd.h
        ndnet_ndt_take_sync_failures).  Every ``run``, ``ndt_preprocessing``
        call and pipeline replay checks it, whatever ``check`` says."""
        rc = _lib.lib().ndnet_ndt_take_sync_failures(self.handle)
        if rc < 0:
            _lib.check(rc, "ndnet_ndt_take_sync_failures")
        if rc:
            raise NdtCloudError([_lib.NDNET_ERR_SYNC], sync=True)

    def prune(self, num_nds: int, out: torch.Tensor, out_classes: Optional[torch.Tensor] = None) -> None:
        st = _lib.stream_ptr(self.device)
        rc = _lib.lib().ndnet_ndt_prune(self.handle, st, num_nds, out.data_ptr(),
                                        out_classes.data_ptr() if out_classes is not None else None,
                                        None, None, None, self.stats.data_ptr())
        _lib.check(rc, "ndnet_ndt_prune")

    def host_stats(self) -> list:
        raw = self.stats.cpu().numpy().tobytes()
        return [_lib.NdtStats.from_buffer_copy(raw, i * _lib.STATS_BYTES) for i in range(self.batch)]


_plans: dict = {}


def get_plan(batch: int, num_points: int, num_nds: int, num_classes: int, device: torch.device) -> NdtPlan:
    key = (batch, num_points, num_nds, num_classes, device)
    p = _plans.get(key)
    if p is None:
        p = NdtPlan(batch, num_points, num_nds, num_classes, device=device)
        _plans[key] = p
    return p


# opt-in failure check of every eager ndt_preprocessing call (see its docstring)
CHECK_RC = os.environ.get("NDNET_CHECK_RC", "0") == "1"


class NdtCloudError(RuntimeError):
    """A cloud of the batch failed (``rcs``: per-cloud return codes)."""

    def __init__(self, rcs, sync: bool = False):
        self.rcs = list(rcs)
        if sync:
            super().__init__("an earlier ndt_downsample run failed: a k_front cloud barrier timed out (rc -22, "
                             "NDNET_ERR_SYNC); its clouds hold zero rows")
            return
        bad = {b: rc for b, rc in enumerate(self.rcs) if rc != 0}
        super().__init__(f"ndt_downsample failed for clouds {bad} (rc -3: search hit 15 iterations, "
                         f"-1: grid above the voxel capacity, -22: front barrier timeout)")


def check_stats(plan: "NdtPlan") -> None:
    """Raises ``NdtCloudError`` if any cloud of the plan's last run failed
    (synchronises with the plan's stream)."""
    rcs = [s.rc for s in plan.host_stats()]
    plan.raise_sync_failures()  # consumed here: the per-cloud codes below carry it
    if any(rc != 0 for rc in rcs):
        raise NdtCloudError(rcs)


def ndt_preprocessing(num_nds: int, points: torch.Tensor, classes: torch.Tensor = None,
                      num_classes: int = None, *, check: Optional[bool] = None
                      ) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """Downsample a batch of clouds to ``num_nds`` normal distributions.

    Args:
        num_nds: NDs per cloud (the reference's ``n_desired_nds``).
        points: ``[B, N, 3]`` float tensor (any device; computed on the GPU).
        classes: optional ``[B, N, num_classes + 1]`` one-hot labels.
        num_classes: number of classes (labels take ``num_classes + 1`` values).

    Returns:
        ``(points [B, num_nds, 3], covariances [B, num_nds, 9], classes one-hot
        [B, num_nds, num_classes + 1] or None)`` float32 on ``points.device``.
        The first two are views of one ``[B, num_nds, 12]`` block, the layout
        the NDTNet kernels read.

    Failures: like the reference (ndt_legacy.py:153 ignores the return code;
    the zero-filled outputs of ndt_legacy.py:126-143 pass through), a failed
    cloud yields all-zero rows and a class-0 one-hot.  Failure modes are the
    reference's (-3: the bisection reached 15 iterations, ndt.c:191-194) plus
    this build's capacities: a bisection grid above the plan's voxel capacity
    (default 2^22 voxels per cloud) fails the cloud with -1 where the
    reference would malloc it.  ``check=True`` (or ``NDNET_CHECK_RC=1``)
    synchronises and raises ``NdtCloudError`` instead; it is skipped while a
    HIP graph is being captured.  Per-cloud codes: ``last_stats()``.  A
    k_front barrier timeout (-22, no reference code) is never silent: it sets
    a flag in host memory and the plan's next call raises ``NdtCloudError``
    whatever ``check`` is (``NdtPlan.raise_sync_failures``).
    """
    _lib.require_gpu()
    src_device = points.device
    dev = src_device if src_device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
    pts = points.to(device=dev, dtype=torch.float32).contiguous()
    B, N, D = pts.shape
    if D != 3:
        raise ValueError(f"points must be [B, N, 3], got {tuple(pts.shape)}")
    labelled = classes is not None
    if labelled and num_classes is None:
        raise ValueError("num_classes is required with classes")
    ncls = int(num_classes) if labelled else -1
    plan = get_plan(B, N, int(num_nds), ncls, dev)
    out = torch.empty((B, num_nds, 12), dtype=torch.float32, device=dev)
    out_cls = None
    labels = None
    if labelled:
        # argmax of the one-hot labels, as ndtnet_preprocessing.py:34 does per cloud
        oh = classes.to(dev)
        if oh.dtype == torch.float32:  # one HIP pass (torch's argmax + int cast: ~160 us at 16 x 100k x 29)
            oh = oh.contiguous()
            labels = torch.empty(oh.shape[:2], dtype=torch.int32, device=dev)
            _lib.check(_lib.lib().ndnet_row_argmax(oh.data_ptr(), oh.shape[0] * oh.shape[1], oh.shape[2],
                                                   labels.data_ptr(), torch.cuda.current_stream(dev).cuda_stream),
                       "ndnet_row_argmax")
        else:
            labels = torch.argmax(oh, dim=2).to(torch.int32).contiguous()
        out_cls = torch.empty((B, num_nds, ncls + 1), dtype=torch.float32, device=dev)
    plan.run(pts, labels, out, out_cls)
    ndt_preprocessing.last_plan = plan
    if (CHECK_RC if check is None else check) and not torch.cuda.is_current_stream_capturing():
        check_stats(plan)
    if src_device != dev:
        out = out.to(src_device)
        out_cls = out_cls.to(src_device) if out_cls is not None else None
    return out[..., :3], out[..., 3:], out_cls


ndt_preprocessing.last_plan = None


def ndt_multiscale(levels, points: torch.Tensor, classes: torch.Tensor = None, num_classes: int = None) -> list:
    """Multi-level NDT of a batch (config C5, tools/train_multiscale.py's
    levels): ``downsample(levels[0])`` then ``prune(levels[i])`` for each
    further, smaller level on the retained KL list -- NDT_Sampler.downsample /
    .prune (ndt_legacy.py:111-240) for every cloud at once, all on the GPU.

    Returns one ``(points [B,k,3], covariances [B,k,9], classes or None)`` per
    level, as ndt_preprocessing does for one level."""
    levels = [int(k) for k in levels]
    if not levels or any(b >= a for a, b in zip(levels, levels[1:])):
        raise ValueError(f"levels must be strictly decreasing, got {levels}")
    p, c, cls = ndt_preprocessing(levels[0], points, classes, num_classes)
    out = [(p, c, cls)]
    plan = ndt_preprocessing.last_plan
    dev = plan.device
    B = p.shape[0]
    for k in levels[1:]:
        blk = torch.empty((B, k, 12), dtype=torch.float32, device=dev)
        blk_cls = torch.empty((B, k, cls.shape[2]), dtype=torch.float32, device=dev) if cls is not None else None
        plan.prune(k, blk, blk_cls)
        if points.device != dev:
            blk = blk.to(points.device)
            blk_cls = blk_cls.to(points.device) if blk_cls is not None else None
        out.append((blk[..., :3], blk[..., 3:], blk_cls))
    return out


def ndt_preprocessing_packed(num_nds: int, points: torch.Tensor) -> torch.Tensor:
    """The unlabelled path returning the ``[B, num_nds, 12]`` block itself."""
    p, _, _ = ndt_preprocessing(num_nds, points)
    return p.as_strided((p.shape[0], p.shape[1], 12), (p.shape[1] * 12, 12, 1))


def last_stats() -> list:
    """Per-cloud ``ndnet_ndt_stats`` of the last ``ndt_preprocessing`` call."""
    plan = ndt_preprocessing.last_plan
    return plan.host_stats() if plan is not None else []
