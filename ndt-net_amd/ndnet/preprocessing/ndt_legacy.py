"""``NDT_Sampler``: the single-cloud sampler of the reference, on the GPU.

Drop-in for ``ndnet.preprocessing.ndt_legacy.NDT_Sampler``
(reference ndnet/preprocessing/ndt_legacy.py:45-240): same constructor,
``downsample(k)``, ``prune(k)`` and ``cleanup()``, same ctypes attributes
(``len_x``/``len_y``/``len_z``, ``offset_*``, ``voxel_size``,
``num_valid_nds``, ``num_kl_divergences``), backed by the reference-ABI entry
points of libndnet_amd.so instead of /usr/local/lib/libndnet.so.
Return codes are no longer ignored: a failed call raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _lib


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class NDT_Sampler:
    """Downsample one point cloud with NDT (voxel NDs + KL prune)."""

    def __init__(self, pointcloud: np.ndarray, classes: np.ndarray = None, num_classes: int = None) -> None:
        self.pointcloud = np.ascontiguousarray(pointcloud, dtype=np.float64)
        self.covariances = None
        self.classes = None if classes is None else np.ascontiguousarray(classes, dtype=np.uint16)
        self.num_classes = int(num_classes) if num_classes is not None else 0
        self.num_points = len(self.pointcloud)
        self.num_valid_nds = ctypes.pointer(ctypes.c_ulong(0))
        self.len_x = ctypes.pointer(ctypes.c_uint(0))
        self.len_y = ctypes.pointer(ctypes.c_uint(0))
        self.len_z = ctypes.pointer(ctypes.c_uint(0))
        self.offset_x = ctypes.pointer(ctypes.c_double(0.0))
        self.offset_y = ctypes.pointer(ctypes.c_double(0.0))
        self.offset_z = ctypes.pointer(ctypes.c_double(0.0))
        self.voxel_size = ctypes.pointer(ctypes.c_double(0.0))
        self.nd_array_ptr = ctypes.c_void_p()
        self.kl_divergences_ptr = ctypes.c_void_p()
        self.num_kl_divergences = ctypes.pointer(ctypes.c_ulong(0))
        self.last_rc = 0
        self.destroyed = False

    # -- lifetime ------------------------------------------------------------
    def cleanup(self) -> None:
        core = _lib.lib()
        core.free_nds(self.nd_array_ptr, self.len_x.contents.value * self.len_y.contents.value
                      * self.len_z.contents.value)
        core.free_kl_divergences(self.kl_divergences_ptr)
        self.nd_array_ptr = ctypes.c_void_p()
        self.kl_divergences_ptr = ctypes.c_void_p()
        self.destroyed = True

    def __del__(self) -> None:
        if not getattr(self, "destroyed", True):
            try:
                self.cleanup()
            except Exception:
                pass

    # -- sampling ------------------------------------------------------------
    def _grid(self):
        return self.len_x.contents.value, self.len_y.contents.value, self.len_z.contents.value

    def downsample(self, num_desired_points: int):
        """Returns ``(points [k,3] f64, covariances [k,9] f64, classes [k] u16)``."""
        _lib.require_gpu()
        k = int(num_desired_points)
        new_pcl = np.zeros((k, 3), dtype=np.float64)
        covs = np.zeros((k, 9), dtype=np.float64)
        new_cls = np.zeros(k, dtype=np.uint16)
        n_out = ctypes.c_ulong(0)
        cls_ptr = None if self.classes is None else self.classes.ctypes.data_as(ctypes.POINTER(ctypes.c_ushort))
        rc = _lib.lib().ndt_downsample(
            _dptr(self.pointcloud), 3, self.num_points,
            self.len_x, self.len_y, self.len_z,
            self.offset_x, self.offset_y, self.offset_z, self.voxel_size,
            cls_ptr, self.num_classes, k,
            _dptr(new_pcl), ctypes.byref(n_out), _dptr(covs),
            new_cls.ctypes.data_as(ctypes.POINTER(ctypes.c_ushort)),
            ctypes.byref(self.nd_array_ptr), self.num_valid_nds,
            ctypes.byref(self.kl_divergences_ptr), self.num_kl_divergences)
        self.last_rc = rc
        if rc != 0:
            raise RuntimeError(f"ndt_downsample failed with code {rc}")
        self.num_points = k
        return new_pcl, covs, new_cls

    def prune(self, new_desired_points: int):
        """Prune the retained NDs further with the KL list of the first level.

        Returns ``(points [k,3] f64, covariances [k,9] f64, classes [k] i16)``:
        the reference allocates the pruned classes as ``np.int16``
        (ndt_legacy.py:211) where ``downsample`` uses ``np.uint16`` (:138)."""
        k = int(new_desired_points)
        core = _lib.lib()
        lx, ly, lz = self._grid()
        rc = core.prune_nds(self.nd_array_ptr, lx, ly, lz, k, self.num_valid_nds,
                            self.kl_divergences_ptr, self.num_kl_divergences)
        self.last_rc = rc
        # -1 (k > valid) and -2 (list exhausted) leave a valid set, which the
        # reference goes on to emit (its return code is ignored, ndt_legacy.py:
        # 194-197); API errors and a walk into never-written entries raise.
        if rc not in (0, -1, -2):
            raise RuntimeError(f"prune_nds failed with code {rc}")
        new_pcl = np.zeros((k, 3), dtype=np.float64)
        covs = np.zeros((k, 9), dtype=np.float64)
        new_cls = np.zeros(k, dtype=np.int16)
        n_out = ctypes.c_ulong(0)
        rc2 = core.to_point_cloud(self.nd_array_ptr, lx, ly, lz, self.offset_x.contents.value,
                                  self.offset_y.contents.value, self.offset_z.contents.value,
                                  self.voxel_size.contents.value, _dptr(new_pcl), ctypes.byref(n_out), _dptr(covs),
                                  new_cls.ctypes.data_as(ctypes.POINTER(ctypes.c_ushort)))
        if rc2 != 0:
            raise RuntimeError(f"to_point_cloud failed with code {rc2}")
        self.num_points = k
        self.pointcloud = new_pcl
        self.covariances = covs
        self.classes = new_cls
        return new_pcl, covs, new_cls
