"""ctypes front-end of the CPU oracle (oracle/ndt_oracle.c) and of the reference
estimate stage compiled into oracle/_ref (oracle/ref_harness.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline, never as
the product path.  The product (ndt-net_amd/) must not import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libref_estimate.so")

_P = ctypes.c_void_p
_U64 = ctypes.c_uint64


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


class _SearchT(ctypes.Structure):
    _fields_ = [
        ("rc", ctypes.c_int),
        ("iters", ctypes.c_int),
        ("guesses", ctypes.c_double * 15),
        ("counts", ctypes.c_uint64 * 15),
        ("lim", ctypes.c_double * 6),
        ("len", ctypes.c_int * 3),
        ("off", ctypes.c_double * 3),
        ("voxel_size", ctypes.c_double),
        ("num_nds", ctypes.c_uint64),
    ]


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        assert _lib.orc_search_struct_size() == ctypes.sizeof(_SearchT)
        _lib.orc_run.restype = ctypes.c_int
        _lib.orc_search.restype = ctypes.c_int
        _lib.orc_portable_log.restype = ctypes.c_double
        _lib.orc_portable_log.argtypes = [ctypes.c_double]
    return _lib


def ref_lib():
    """The reference's estimate stage (None when oracle/_ref was not built)."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB):
        _ref = ctypes.CDLL(REF_LIB)
    return _ref


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def set_portable_log(on: bool) -> None:
    ctypes.c_int.in_dll(lib(), "orc_use_portable_log").value = 1 if on else 0


def set_gsl_invert(on: bool) -> None:
    """1: gsl_linalg_LU_invert as GSL 2.7.1 publishes it (default);
    0: the column-solve variant (A/B comparisons only)."""
    ctypes.c_int.in_dll(lib(), "orc_use_gsl_invert").value = 1 if on else 0


@dataclass
class SearchResult:
    rc: int
    guesses: np.ndarray
    counts: np.ndarray
    lim: np.ndarray
    len: tuple
    off: np.ndarray
    voxel_size: float
    num_nds: int


def _search_result(s: _SearchT) -> SearchResult:
    it = s.iters
    return SearchResult(
        rc=s.rc,
        guesses=np.array(s.guesses[:it]),
        counts=np.array(s.counts[:it], dtype=np.uint64),
        lim=np.array(s.lim[:]),
        len=tuple(s.len[:]),
        off=np.array(s.off[:]),
        voxel_size=s.voxel_size,
        num_nds=s.num_nds,
    )


def search(points: np.ndarray, k: int) -> SearchResult:
    pts = np.ascontiguousarray(points, dtype=np.float64)
    s = _SearchT()
    lib().orc_search(_ptr(pts), 3, _U64(len(pts)), _U64(k), ctypes.byref(s))
    return _search_result(s)


@dataclass
class RunResult:
    rc: int
    search: SearchResult
    vox_n: np.ndarray = field(default=None)
    vox_mean: np.ndarray = field(default=None)
    vox_cov_pre: np.ndarray = field(default=None)
    vox_cov_post: np.ndarray = field(default=None)
    vox_cls: np.ndarray = field(default=None)
    vox_kept: np.ndarray = field(default=None)
    ev_div: np.ndarray = field(default=None)
    ev_p: np.ndarray = field(default=None)
    ev_q: np.ndarray = field(default=None)
    ev_rc: np.ndarray = field(default=None)
    ord_div: np.ndarray = field(default=None)
    ord_p: np.ndarray = field(default=None)
    ord_q: np.ndarray = field(default=None)
    prune_rc: int = 0
    num_valid: int = 0
    out_pc: np.ndarray = field(default=None)
    out_cov: np.ndarray = field(default=None)
    out_cls: np.ndarray = field(default=None)
    nout: int = 0
    post_div: np.ndarray = field(default=None)
    post_p: np.ndarray = field(default=None)
    post_q: np.ndarray = field(default=None)
    post_nkl: int = 0


def run(points: np.ndarray, k: int, classes: np.ndarray | None = None, num_classes: int = 0,
        portable_log: bool = True) -> RunResult:
    """The whole ndt_downsample path with every stage exposed."""
    set_portable_log(portable_log)
    pts = np.ascontiguousarray(points, dtype=np.float64)
    n = len(pts)
    cls = None if classes is None else np.ascontiguousarray(classes, dtype=np.uint16)
    pre = search(pts, k)
    if pre.rc < 0:
        return RunResult(rc=pre.rc, search=pre)
    V = int(np.prod(pre.len))
    vcap, ecap = max(V, 1), max(6 * V, 1)
    r = RunResult(rc=0, search=pre)
    r.vox_n = np.zeros(vcap, np.uint64)
    r.vox_mean = np.zeros((vcap, 3))
    r.vox_cov_pre = np.zeros((vcap, 9))
    r.vox_cov_post = np.zeros((vcap, 9))
    r.vox_cls = np.zeros(vcap, np.uint16)
    r.vox_kept = np.zeros(vcap, np.uint8)
    r.ev_div = np.zeros(ecap)
    r.ev_p = np.zeros(ecap, np.int64)
    r.ev_q = np.zeros(ecap, np.int64)
    r.ev_rc = np.zeros(ecap, np.int32)
    r.ord_div = np.zeros(ecap)
    r.ord_p = np.zeros(ecap, np.int64)
    r.ord_q = np.zeros(ecap, np.int64)
    r.out_pc = np.zeros((k, 3))
    r.out_cov = np.zeros((k, 9))
    r.out_cls = np.zeros(k, np.uint16)
    r.post_div = np.zeros(ecap)
    r.post_p = np.zeros(ecap, np.int64)
    r.post_q = np.zeros(ecap, np.int64)
    s = _SearchT()
    nvox, nev, nord, nout, nvalid, pnkl = (_U64(0) for _ in range(6))
    prc = ctypes.c_int(0)
    rc = lib().orc_run(
        _ptr(pts), _U64(n), _ptr(cls), ctypes.c_int(num_classes), _U64(k), ctypes.byref(s), _U64(vcap),
        _ptr(r.vox_n), _ptr(r.vox_mean), _ptr(r.vox_cov_pre), _ptr(r.vox_cov_post), _ptr(r.vox_cls),
        _ptr(r.vox_kept), _U64(ecap), _ptr(r.ev_div), _ptr(r.ev_p), _ptr(r.ev_q), _ptr(r.ev_rc),
        _ptr(r.ord_div), _ptr(r.ord_p), _ptr(r.ord_q), ctypes.byref(nvox), ctypes.byref(nev), ctypes.byref(nord),
        ctypes.byref(prc), ctypes.byref(nvalid), _ptr(r.out_pc), _ptr(r.out_cov), _ptr(r.out_cls),
        ctypes.byref(nout), _ptr(r.post_div), _ptr(r.post_p), _ptr(r.post_q), ctypes.byref(pnkl))
    r.rc = rc
    r.search = _search_result(s)
    e = nev.value
    r.ev_div, r.ev_p, r.ev_q, r.ev_rc = r.ev_div[:e], r.ev_p[:e], r.ev_q[:e], r.ev_rc[:e]
    o = nord.value
    r.ord_div, r.ord_p, r.ord_q = r.ord_div[:o], r.ord_p[:o], r.ord_q[:o]
    r.post_div, r.post_p, r.post_q = r.post_div[:o], r.post_p[:o], r.post_q[:o]
    r.post_nkl = pnkl.value
    r.prune_rc = prc.value
    r.num_valid = nvalid.value
    r.nout = nout.value
    return r


def downsample_f32(points: np.ndarray, k: int, portable_log: bool = True):
    """What ndt_preprocessing yields for one cloud: [k,3] and [k,9] float32 after
    nan_to_num (ndtnet_preprocessing.py:30-67), plus the return code."""
    r = run(points, k, portable_log=portable_log)
    pc = np.zeros((k, 3), np.float32)
    cov = np.zeros((k, 9), np.float32)
    if r.rc == 0:
        pc = np.nan_to_num(r.out_pc.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
        cov = np.nan_to_num(r.out_cov.astype(np.float32), nan=0.0, posinf=0.0, neginf=0.0)
    return pc, cov, r


# ---------------- the reference's own estimate stage (oracle/_ref) ----------------

def ref_limits(points: np.ndarray) -> np.ndarray:
    pts = np.ascontiguousarray(points, dtype=np.float64)
    lim = np.zeros(6)
    ref_lib().ref_limits(_ptr(pts), ctypes.c_short(3), ctypes.c_ulong(len(pts)), _ptr(lim))
    return lim


def ref_estimate(points: np.ndarray, voxel_size: float, length, offset, classes=None, num_classes=0,
                 threads: bool = False):
    pts = np.ascontiguousarray(points, dtype=np.float64)
    ln = np.array(length, dtype=np.int32)
    off = np.array(offset, dtype=np.float64)
    V = int(np.prod(ln.astype(np.int64)))
    cnt = np.zeros(max(V, 1), np.uint64)
    mean = np.zeros((max(V, 1), 3))
    cov = np.zeros((max(V, 1), 9))
    cls_out = np.zeros(max(V, 1), np.uint16)
    cls = None if classes is None else np.ascontiguousarray(classes, dtype=np.uint16)
    nn = _U64(0)
    fn = ref_lib().ref_estimate_threads if threads else ref_lib().ref_estimate_seq
    rc = fn(_ptr(pts), ctypes.c_ulong(len(pts)), _ptr(cls), ctypes.c_ushort(num_classes),
            ctypes.c_double(voxel_size), _ptr(ln), _ptr(off), _ptr(cnt), _ptr(mean), _ptr(cov),
            _ptr(cls_out), ctypes.byref(nn))
    assert rc == 0
    return cnt[:V], mean[:V], cov[:V], cls_out[:V], nn.value


def ref_search(points: np.ndarray, k: int):
    pts = np.ascontiguousarray(points, dtype=np.float64)
    g = np.zeros(15)
    c = np.zeros(15, np.uint64)
    it = ctypes.c_int(0)
    ln = np.zeros(3, np.int32)
    off = np.zeros(3)
    vs = ctypes.c_double(0)
    rc = ref_lib().ref_search(_ptr(pts), ctypes.c_ulong(len(pts)), ctypes.c_ulong(k), _ptr(g), _ptr(c),
                              ctypes.byref(it), _ptr(ln), _ptr(off), ctypes.byref(vs))
    return rc, g[:it.value], c[:it.value], tuple(ln), off, vs.value


class LegacyChain:
    """The oracle's implementation of the reference ABI driven like
    NDT_Sampler (ndt_legacy.py:111-240): downsample, then prune levels."""

    def __init__(self, points: np.ndarray, portable_log: bool = True):
        set_portable_log(portable_log)
        self.pts = np.ascontiguousarray(points, dtype=np.float64)
        self.L = lib()
        self.lx, self.ly, self.lz = ctypes.c_uint(0), ctypes.c_uint(0), ctypes.c_uint(0)
        self.ox, self.oy, self.oz, self.vs = (ctypes.c_double(0) for _ in range(4))
        self.nd = ctypes.c_void_p()
        self.kl = ctypes.c_void_p()
        self.nvalid = ctypes.c_ulong(0)
        self.nkl = ctypes.c_ulong(0)
        self.rc = 0

    def downsample(self, k: int):
        pc = np.zeros((k, 3))
        cov = np.zeros((k, 9))
        cls = np.zeros(k, np.uint16)
        nout = ctypes.c_ulong(0)
        self.rc = self.L.ndt_downsample(
            _ptr(self.pts), ctypes.c_ushort(3), ctypes.c_ulong(len(self.pts)), ctypes.byref(self.lx),
            ctypes.byref(self.ly), ctypes.byref(self.lz), ctypes.byref(self.ox), ctypes.byref(self.oy),
            ctypes.byref(self.oz), ctypes.byref(self.vs), None, ctypes.c_ushort(0), ctypes.c_ulong(k), _ptr(pc),
            ctypes.byref(nout), _ptr(cov), _ptr(cls), ctypes.byref(self.nd), ctypes.byref(self.nvalid),
            ctypes.byref(self.kl), ctypes.byref(self.nkl))
        return pc, cov

    def prune(self, k: int):
        self.rc = self.L.prune_nds(self.nd, self.lx, self.ly, self.lz, ctypes.c_ulong(k), ctypes.byref(self.nvalid),
                                   self.kl, ctypes.byref(self.nkl))
        pc = np.zeros((k, 3))
        cov = np.zeros((k, 9))
        cls = np.zeros(k, np.uint16)
        nout = ctypes.c_ulong(0)
        # the oracle's to_point_cloud has no capacity either: give it room, then keep k rows
        big = max(int(self.nvalid.value), k)
        pcb = np.zeros((big, 3))
        covb = np.zeros((big, 9))
        clsb = np.zeros(big, np.uint16)
        self.L.to_point_cloud(self.nd, self.lx, self.ly, self.lz, self.ox, self.oy, self.oz, self.vs, _ptr(pcb),
                              ctypes.byref(nout), _ptr(covb), _ptr(clsb))
        m = min(k, int(nout.value))
        pc[:m], cov[:m], cls[:m] = pcb[:m], covb[:m], clsb[:m]
        return pc, cov

    def cleanup(self):
        self.L.free_nds(self.nd, ctypes.c_ulong(self.lx.value * self.ly.value * self.lz.value))
        self.L.free_kl_divergences(self.kl)
        self.nd = ctypes.c_void_p()
        self.kl = ctypes.c_void_p()


# ---------------- the reference-structured CPU baseline (oracle/cpu_ref.c) ----------------

CPUREF_LIB = os.path.join(HERE, "libcpu_ref.so")
_cref = None


def cref_lib():
    global _cref
    if _cref is None:
        if not os.path.exists(CPUREF_LIB):
            build()
        _cref = ctypes.CDLL(CPUREF_LIB)
        _cref.cref_downsample.restype = ctypes.c_int
        _cref.cref_estimate_only.restype = ctypes.c_int
    return _cref


def cref_downsample(points: np.ndarray, k: int):
    """One ndt_downsample through the reference-structured baseline (8
    pthreads, mutex per voxel, GSL-style heap traffic, -O0): rows and rc."""
    pts = np.ascontiguousarray(points, dtype=np.float64)
    pc, cov = np.zeros((k, 3)), np.zeros((k, 9))
    nout = _U64(0)
    rc = cref_lib().cref_downsample(_ptr(pts), _U64(len(pts)), _U64(k), _ptr(pc), _ptr(cov), ctypes.byref(nout))
    return pc, cov, rc


def cref_estimate_only(points: np.ndarray, voxel_size: float, length, offset) -> int:
    pts = np.ascontiguousarray(points, dtype=np.float64)
    ln = np.array(length, dtype=np.int32)
    off = np.array(offset, dtype=np.float64)
    nn = _U64(0)
    rc = cref_lib().cref_estimate_only(_ptr(pts), _U64(len(pts)), ctypes.c_double(voxel_size), _ptr(ln), _ptr(off),
                                       ctypes.byref(nn))
    assert rc == 0
    return nn.value


def legacy_downsample_rows(points: np.ndarray, k: int) -> int:
    """One oracle ndt_downsample through its legacy ABI (the lightest call:
    k output rows, handles freed at once); returns the reference's code.
    The ctypes call releases the GIL, so threads run clouds in parallel."""
    pts = np.ascontiguousarray(points, dtype=np.float64)
    ch = LegacyChain.__new__(LegacyChain)
    ch.pts, ch.L = pts, lib()
    ch.lx, ch.ly, ch.lz = ctypes.c_uint(0), ctypes.c_uint(0), ctypes.c_uint(0)
    ch.ox, ch.oy, ch.oz, ch.vs = (ctypes.c_double(0) for _ in range(4))
    ch.nd, ch.kl = ctypes.c_void_p(), ctypes.c_void_p()
    ch.nvalid, ch.nkl, ch.rc = ctypes.c_ulong(0), ctypes.c_ulong(0), 0
    ch.downsample(k)
    rc = ch.rc
    ch.cleanup()
    return rc
