"""NDT preprocessing + NDTNetSegmentation eval forward as one HIP graph.

The reference runs ``ndt_preprocessing`` then ``model(points, covariances)``
per batch (ndnet/train_segmentation.py / ndnet/models/ndtnet.py:218-243), with
a host round trip per cloud in between.  Here both halves are GPU-resident
and launch ~45 kernels per batch (17 NDT launches, 4 point-MLP chains, the
per-cloud FC heads / weight folds); on a 1 ms step the host-side launch cost
of that sequence is a large fraction of the step.  ``GraphedSegmentation``
captures the whole sequence once into a HIP graph (``torch.cuda.CUDAGraph``
is hipGraph on ROCm) and replays it: every kernel still runs on every step,
only the host launch work is gone.

Capture is legal because neither half synchronises or allocates device
memory after its first (warm-up) call: the NDT plan and the forward's
workspace are cached per shape, and the NDT stamp-epoch wrap is handled on
the device (k_reset / k_limits), not by host bookkeeping.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import _lib
from .preprocessing.ndtnet_preprocessing import NdtPlan, ndt_multiscale, ndt_preprocessing, get_plan


# CU share of the pipelined NDT stage (ndnet_ndt_set_cu_share): k_front and
# k_welford_q take CUs / share, leaving the rest to the forward's kernels on
# the other stream.  Measured on C2 (profiles/r03n_cu_share.txt): share 2
# 69.8k clouds/s against 64.1k at share 1, although the NDT stage alone
# slows from 100 to 136 us -- at share 1 k_front needs every CU at once and
# the two streams serialise.
PIPE_CU_SHARE = int(os.environ.get("NDNET_PIPE_CU_SHARE", "2"))
# k_welford_q keeps every CU: front 2 / welford 1 measured 70.5k clouds/s
# against 68.8-70.2k for 2 / 2 and 62.8k for 2 / 4 (profiles/r03n_cu_share.txt)
PIPE_WQ_SHARE = int(os.environ.get("NDNET_PIPE_WQ_SHARE", "1"))
# ... and of a pipeline with more than one NDT stream (the L clouds' two):
# share 3 measured 67.8 / 68.0k against 67.3 / 67.2k clouds/s at 2 and 67.4k
# at 4 on one box, 66.3 / 66.1k against 66.1 / 66.3k on another (+0.5% over
# both, within the spread; profiles/r06sl_cu_share_ab.txt), where the U line
# keeps 2 (88.3k; 3: 87.7-89.1k, 4: 87.4k)
PIPE_CU_SHARE_MULTI = int(os.environ.get("NDNET_PIPE_CU_SHARE_MULTI", "3"))
# Forward streams of PipelinedSegmentation: more than one lets consecutive
# forwards overlap (each in its own workspace slot), one's TNet heads and
# chain prologues beside the other's chains.  C2: 1 stream 74.9-75.0k, 2
# streams 74.8-78.8k, 3 streams (default) 81.7k clouds/s; C5 20.7k -> 23.7-24.4k
# with 2 or 3 (profiles/r03aa_fwd_streams.txt, r03ab_fwd_streams.txt).  With the
# NDT stream that is 4 streams, the hardware queues a process gets by default.
PIPE_FWD_STREAMS = int(os.environ.get("NDNET_PIPE_FWD_STREAMS", "3"))
# NDT streams, each with its own plan (workspace): 2 lets the NDT stage of
# consecutive batches overlap, for clouds whose NDT stage outlasts a forward
# (L: k_welford_q's heaviest ND alone takes ~90 us).  Measured: L 47.6k ->
# 53.2k clouds/s, but U 83k -> 79k and C5 26.0k -> 25.7k, so 1 by default
# (profiles/r03ah_ndt_streams.txt)
PIPE_NDT_STREAMS = int(os.environ.get("NDNET_PIPE_NDT_STREAMS", "1"))
# k_welford_q's light form for the plans of a pipeline with more than one NDT
# stream ("quad", "light64" or "auto": by the CU share, light64 here)
PIPE_WQ_FORM_MULTI = os.environ.get("NDNET_PIPE_WQ_FORM_MULTI", "quad")
# Stream priorities: "none" (default), "fwd" (the forward streams high, so the
# TNet heads' few workgroups are dispatched ahead of k_front / chain
# workgroups queued on the other streams) or "ndt".  Measured
# (profiles/r04_priority_ab.txt): none 83.6k, fwd 71.5k, ndt 79.9k clouds/s.
PIPE_PRIORITY = os.environ.get("NDNET_PIPE_PRIORITY", "none")


class _Pinned:
    """What a captured graph reads through raw pointers, kept alive for the
    graph's lifetime: the model's folded-weight cache (weights, workspace,
    prebuilt argument blocks) and the NDT plans.

    Captured graphs follow the model's weights (one behaviour,
    whatever changed them).  ``check()`` runs before every replay: when a
    weight changed since the last fold -- an in-place update, an optimizer
    step, ``model.train()`` then ``eval()`` around a replayed training graph
    that changes weights without bumping their versions -- it re-folds in
    place (one ``ndnet_pn_fold_run`` launch on the caller's stream: after the
    previous replays, which the caller's stream has joined, and before this
    one, whose streams fork from it), so the replay computes with the current
    weights.  A fold that cannot be redone in place (a parameter tensor
    replaced, a dtype change) leaves the graph pointing at the old buffers:
    the replay raises, and a new graph must be built."""

    def __init__(self, model, plans) -> None:
        from .models import pointnet_hip
        self.model, self.plans = model, list(plans)
        self.cache = model._hip
        if self.cache is None or "W" not in self.cache:
            raise RuntimeError("the capture ran no HIP forward (is the HIP path built?)")
        self.W, self.ws, self.sig = self.cache["W"], dict(self.cache["ws"]), self.cache["sig"]
        self._signature = lambda: pointnet_hip._signature(self.cache["tensors"])

    def check(self) -> None:
        from .models import pointnet_hip
        for plan in self.plans:  # a k_front barrier timeout of an earlier replay (no sync)
            plan.raise_sync_failures()
        if self.model.training:
            raise RuntimeError("replaying an eval-mode graph with the model in train mode: call model.eval()")
        cur = pointnet_hip._tensors(self.model)
        same = len(cur) == len(self.cache["tensors"]) and all(a is b for a, b in zip(cur, self.cache["tensors"]))
        if same and self.cache.get("W") is self.W and self._signature() == self.sig and not self.cache.get("stale"):
            return
        pointnet_hip._folded(self.model)  # re-folds in place when it can
        if self.cache.get("W") is not self.W:
            raise RuntimeError("the model's weights changed after the graph was captured in a way the fold "
                               "cannot follow in place (a parameter replaced?): build a new graph")
        self.sig = self.cache["sig"]


class GraphedSegmentation:
    """Replays ``model(*ndt_preprocessing(num_nds, points)[:2])`` from a graph.

    Args:
        model: an ``NDTNetSegmentation`` in eval mode on a cuda device.  Its
            weights are folded at capture time; the replays follow later
            in-place weight changes (re-folded before the replay, see
            ``_Pinned``); a replaced parameter tensor makes the replay raise.
        num_nds: NDs per cloud (the reference's ``n_desired_nds``).
        batch, num_points: the static input shape ``[batch, num_points, 3]``.
        warmup: eager runs before capture (plan / workspace creation, kernel
            attribute setup).
        levels: optional strictly decreasing NDs per level (config C5:
            (2000, 1000, 500)): the step is then ndt_multiscale (downsample to
            levels[0], prune to each further level) and a forward per level;
            the output is the list of per-level log-probs.

    ``points`` is the static float32 input buffer; ``__call__(new_points)``
    copies into it, replays, and returns the static ``[B, num_nds, C+1]``
    output buffer (overwritten by the next replay -- clone to keep it).
    """

    def __init__(self, model, num_nds: int, batch: int, num_points: int,
                 device: Optional[torch.device] = None, warmup: int = 2, levels=None) -> None:
        _lib.require_gpu()
        if model.training:
            raise ValueError("GraphedSegmentation needs an eval-mode model")
        dev = torch.device(device) if device is not None else next(model.parameters()).device
        if dev.type != "cuda":
            raise ValueError("GraphedSegmentation needs the model on a cuda device")
        self.levels = tuple(int(k) for k in levels) if levels else None
        if self.levels:
            num_nds = self.levels[0]
        self.model, self.num_nds, self.device = model, int(num_nds), dev
        self.points = torch.zeros((batch, num_points, 3), dtype=torch.float32, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self._step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = self._step()
        self.plan = get_plan(batch, num_points, self.num_nds, -1, dev)
        self._pinned = _Pinned(model, [self.plan])

    def _step(self):
        if self.levels:
            return [self.model(p, c) for p, c, _ in ndt_multiscale(self.levels, self.points)]
        p, c, _ = ndt_preprocessing(self.num_nds, self.points)
        return self.model(p, c)

    def replay(self) -> torch.Tensor:
        self._pinned.check()
        self.graph.replay()
        return self.out

    def __call__(self, points: Optional[torch.Tensor] = None) -> torch.Tensor:
        if points is not None:
            self.points.copy_(points, non_blocking=True)
        return self.replay()

    def stats(self) -> list:
        """Per-cloud ``ndnet_ndt_stats`` of the last replay (synchronises)."""
        return self.plan.host_stats()


class PipelinedSegmentation:
    """Two-stage pipeline over consecutive batches: step i runs the NDT stage
    of batch i on one stream while the forward of batch i - 1 runs on
    another, over a ring of R = 3 input / row buffers.

    The NDT stage is latency-bound (dependent bisection passes with chip-level
    barriers, one-workgroup-per-cloud prune walks, small KL launches) and the
    forward is MFMA-bound, so the two overlap on the GPU; every step still
    runs the whole NDT of one batch and the whole forward of one batch.  The
    forward of step i returns the log-probs of the batch of step i - 1 (the
    first step's forward runs on the warm-up batch).

    Each stage of each ring slot is its own HIP graph, captured on its own
    stream (``g_ndt[j]`` on the NDT stream, ``g_fwd[j]`` on the forward
    stream).  Step i (slot j = i % R) reads input j, writes rows j, and its
    forward reads rows j - 1.  The streams are ordered by events only: the
    forward of step i waits for the NDT of step i - 1 (the rows it reads), the
    NDT of step i for the forward of step i - 2 (the last reader of the rows
    it overwrites).  ``replay()`` runs one step joined with the caller's
    stream at both ends (its output is ready in stream order);
    ``replay_steps(k)`` runs k steps joined only at the ends, so the NDT
    stream runs up to a step ahead of the forward stream and no per-step
    join separates the graphs.  (Round 3 recorded a crash capturing several
    steps in one graph; round 4 found every such capture form working or
    failing cleanly, profiles/r04_capture_probe.txt: a multi-step graph would
    end in a join of every stream, which the per-stage graphs avoid.)

    ``points`` is the buffer the NEXT step reads (fill it, then replay);
    ``load_resident(pts)`` fills every buffer.  ``replay_streamed(host_next)``
    replays the next step and, on a copy stream overlapped with it, copies
    ``host_next`` (pinned host memory) into the buffer of the step after it --
    the PCIe-inclusive serving loop.

    ``levels`` (config C5): the NDT stage is ndt_multiscale (downsample to
    levels[0], prune to each further level) and the forward stage one forward
    per level; the output is then the list of per-level log-probs.
    """

    def __init__(self, model, num_nds: int, batch: int, num_points: int,
                 device: Optional[torch.device] = None, warmup: int = 2, cu_share: Optional[int] = None,
                 levels=None, fwd_streams: Optional[int] = None, ndt_streams: Optional[int] = None) -> None:
        _lib.require_gpu()
        if model.training:
            raise ValueError("PipelinedSegmentation needs an eval-mode model")
        dev = torch.device(device) if device is not None else next(model.parameters()).device
        self.levels = tuple(int(k) for k in levels) if levels else None
        if self.levels:
            if any(b >= a for a, b in zip(self.levels, self.levels[1:])):
                raise ValueError(f"levels must be strictly decreasing, got {self.levels}")
            num_nds = self.levels[0]
        self.model, self.num_nds, self.device = model, int(num_nds), dev
        # F forward streams: step i's forward runs on stream i % F in workspace
        # slot i % F; N NDT streams: step i's NDT stage on stream i % N with
        # plan i % N.  A ring of R >= F + N + 1 buffers (a multiple of F and N)
        # keeps the rows of every forward in flight apart from those the NDT
        # streams write
        self.F = F = max(1, int(fwd_streams if fwd_streams is not None else PIPE_FWD_STREAMS))
        self.N = N = max(1, int(ndt_streams if ndt_streams is not None else PIPE_NDT_STREAMS))
        lcm = F * N // math.gcd(F, N)
        self.R = R = -(-(F + N + 1) // lcm) * lcm
        self.inputs = [torch.zeros((batch, num_points, 3), dtype=torch.float32, device=dev) for _ in range(R)]
        self.rows = [[torch.zeros((batch, k, 12), dtype=torch.float32, device=dev)
                      for k in (self.levels or (self.num_nds,))] for _ in range(R)]
        # plans of its own (not ndt_preprocessing's cached one): their CU share
        # is a property of the pipeline
        self.plans = [NdtPlan(batch, num_points, self.num_nds, -1, device=dev) for _ in range(N)]
        self.plan = self.plans[0]
        if cu_share is None:
            cu_share = PIPE_CU_SHARE if N == 1 else PIPE_CU_SHARE_MULTI
        # k_front's workgroups of a cloud meet at cloud barriers, so all of them
        # must be resident at once.  One NDT stream: k_front alone spans at most
        # the chip (the other kernels never wait on anything, so they drain).
        # N NDT streams run N k_front launches at once: each must take at most
        # CUs / N, or their resident halves wait on each other until the
        # barrier timeout fails the clouds (measured: 640 ms per step with two
        # streams at share 1).  So the share is at least N, the largest that
        # fits from the requested one down to N; a shape that fits none of them
        # takes the one-launch-per-stage path (no cloud barriers).  With one
        # NDT stream a share the shape does not fit falls back to the largest
        # smaller one that does (at worst share 1: the whole chip).
        self.front_share = []
        for plan in self.plans:
            applied = 1
            if plan.path == 2:
                want = list(range(cu_share, 1, -1)) if N == 1 else list(range(max(cu_share, N), N - 1, -1))
                for sh in want:
                    if sh <= 1:
                        break
                    try:
                        plan.set_cu_share(sh, PIPE_WQ_SHARE)
                        applied = sh
                        break
                    except RuntimeError:  # k_front does not fit that share for this shape
                        continue
                if N > 1 and applied < N:
                    plan.set_path(1)
                    applied = 0
            self.front_share.append(applied)  # 0: the one-launch-per-stage path
            if N > 1 and PIPE_WQ_FORM_MULTI != "auto":
                # two NDT streams (the L clouds' pipeline): k_welford_q's lane-quad
                # form, not light64 -- L 66.0k vs 65.1k clouds/s, while one NDT
                # stream keeps light64 (U 89.2k vs 87.3k with quads):
                # profiles/r06j_welford_form_ab.txt
                plan.set_welford_form(PIPE_WQ_FORM_MULTI)
        # stream priorities (NDNET_PIPE_PRIORITY): none by default, see PIPE_PRIORITY
        hi = torch.cuda.Stream.priority_range()[1] if PIPE_PRIORITY != "none" else 0
        self.s_ndts = [torch.cuda.Stream(device=dev, priority=hi if PIPE_PRIORITY == "ndt" else 0) for _ in range(N)]
        self.s_fwds = [torch.cuda.Stream(device=dev, priority=hi if PIPE_PRIORITY == "fwd" else 0) for _ in range(F)]
        self.s_copy = torch.cuda.Stream(device=dev)
        self.ndt_done = [torch.cuda.Event() for _ in range(R)]  # NDT of slot j finished (rows j, input j free)
        self.fwd_done = [torch.cuda.Event() for _ in range(R)]  # forward of slot j finished (rows j - 1 free)
        self.copied = [torch.cuda.Event() for _ in range(R)]    # input j holds the streamed batch
        self._fork()
        with torch.no_grad():  # plan / workspace creation, kernel attributes
            for i in range(max(R, warmup)):
                with torch.cuda.stream(self.s_ndts[i % R % N]):
                    self._ndt(i % R)
                with torch.cuda.stream(self.s_fwds[i % R % F]):
                    self._fwd(i % R)
        torch.cuda.synchronize(dev)
        self.g_ndt, self.g_fwd, self.out = [], [], []
        for j in range(R):
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g, stream=self.s_ndts[j % N]):
                self._ndt(j)
            self.g_ndt.append(g)
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g, stream=self.s_fwds[j % F]):
                self.out.append(self._fwd(j))
            self.g_fwd.append(g)
        torch.cuda.synchronize(dev)
        self._pinned = _Pinned(model, self.plans)
        self.i = 0

    def _ndt(self, j: int) -> None:
        """The NDT stage of ring slot j on the current stream, with plan j % N."""
        rows, plan = self.rows[j], self.plans[j % self.N]
        plan.run(self.inputs[j], None, rows[0], None)
        for k, blk in zip(self.levels[1:] if self.levels else (), rows[1:]):
            plan.prune(k, blk)

    def _fwd(self, j: int):
        """The forward stage of ring slot j: the rows of slot j - 1, in
        workspace slot j % F (forwards on different streams run concurrently)."""
        from .models import pointnet_hip
        with pointnet_hip.workspace_slot(j % self.F):
            outs = [self.model(r[..., :3], r[..., 3:]) for r in self.rows[(j - 1) % self.R]]
        return outs if self.levels else outs[0]

    def _enqueue(self) -> int:
        """Launches the next step's two graphs, ordered by events only."""
        R, j = self.R, self.i % self.R
        s_fwd = self.s_fwds[j % self.F]
        s_fwd.wait_event(self.ndt_done[(j - 1) % R])         # its rows: the previous step's NDT
        with torch.cuda.stream(s_fwd):
            self.g_fwd[j].replay()
        self.fwd_done[j].record(s_fwd)
        # rows j: last read by the forward of step i - R + 1
        s_ndt = self.s_ndts[j % self.N]
        s_ndt.wait_event(self.fwd_done[(j + 1) % R])
        s_ndt.wait_event(self.copied[j])                    # no-op unless a streamed copy targets input j
        with torch.cuda.stream(s_ndt):
            self.g_ndt[j].replay()
        self.ndt_done[j].record(s_ndt)
        self.i += 1
        return j

    def _fork(self) -> None:
        cur = torch.cuda.current_stream(self.device)
        for st in self.s_ndts + self.s_fwds:
            st.wait_stream(cur)

    def _join(self, j: int) -> None:
        """The caller's stream waits for the last N NDT stages and the last F forwards."""
        cur = torch.cuda.current_stream(self.device)
        for t in range(self.F):
            cur.wait_event(self.fwd_done[(j - t) % self.R])
        for t in range(self.N):
            cur.wait_event(self.ndt_done[(j - t) % self.R])

    @property
    def points(self) -> torch.Tensor:
        """The input buffer the next step reads."""
        return self.inputs[self.i % self.R]

    def load_resident(self, points: torch.Tensor) -> None:
        """Fill every input buffer (every later step re-reads this batch)."""
        for buf in self.inputs:
            buf.copy_(points)

    def replay(self):
        """One step, ordered after the caller's stream and before its later work."""
        self._pinned.check()
        self._fork()
        j = self._enqueue()
        self._join(j)
        return self.out[j]

    def replay_steps(self, k: int):
        """k steps with the streams joined to the caller's only at the ends;
        returns the last step's output."""
        self._pinned.check()
        self._fork()
        j = None
        for _ in range(k):
            j = self._enqueue()
        if j is None:
            return None
        self._join(j)
        return self.out[j]

    def replay_streamed(self, host_next: torch.Tensor):
        """``replay()`` with the H2D copy of the batch after it overlapped."""
        nxt = (self.i + 1) % self.R
        out = self.replay()
        # input nxt: last read by the NDT of step i + 1 - R, finished before this step's join
        self.s_copy.wait_event(self.ndt_done[nxt])
        with torch.cuda.stream(self.s_copy):
            self.inputs[nxt].copy_(host_next, non_blocking=True)
            self.copied[nxt].record(self.s_copy)
        return out

    def stats(self) -> list:
        return self.plan.host_stats()
