#!/usr/bin/env python3
"""Round 4: reproduce / bisect the round-3 crash of ONE HIP graph holding
several unrolled pipelined steps (profiles/r03t_pipeline.txt:38-41).

Each mode runs in its own child process (a host segfault ends only that
child); the parent prints one line per mode.  Modes (2 unrolled steps each,
the pipeline's ring, plans, workspace slots and events):
  serial   one stream: ndt(j), fwd(j), ndt(j+1), fwd(j+1) in the capture stream
  fork     NDT on the capture stream, each forward on a forward stream forked
           from it by an event and joined back before the capture ends
  events   the pipeline's own pattern: NDT and forward streams both forked,
           every cross-stream order by events recorded inside the capture,
           every side stream joined back before the capture ends
  unjoined as `events` but one forward stream is left unjoined (illegal:
           capture end must fail cleanly with an error, not crash)
  subgraph the step replays the per-stage graphs (hipGraphLaunch inside a
           capture)
Every capturing mode is replayed and checked against an eager run of the same
two steps.

    python tools/capture_probe.py [mode ...]
"""
import faulthandler
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ndt-net_amd"))
MODES = ["serial", "fork", "events", "subgraph", "unjoined"]


def child(mode: str) -> None:
    faulthandler.enable()
    import torch
    from ndnet.models.ndtnet import NDTNetSegmentation
    from ndnet.pipeline import PipelinedSegmentation
    from ndnet.synthetic import make_batch
    dev = torch.device("cuda", 0)
    B, n, k = 4, 20_000, 200
    torch.manual_seed(0)
    model = NDTNetSegmentation(3, 28, 768).to(dev).eval()
    pipe = PipelinedSegmentation(model, k, B, n, device=dev)
    for j in range(pipe.R):
        pipe.inputs[j].copy_(torch.from_numpy(make_batch("U" if j % 2 else "L", B, n, seed0=10 * j)).to(dev))
    R, F = pipe.R, pipe.F
    # eager reference of steps j = 1, 2: NDT(j) then forward(j) (reads rows j - 1)
    with torch.no_grad():
        for j in (0, 1, 2):
            pipe._ndt(j)
        ref = [pipe._fwd(j).clone() for j in (1, 2)]
        torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    ev = [torch.cuda.Event() for _ in range(16)]
    outs = []
    print(f"[{mode}] capturing", flush=True)
    with torch.no_grad(), torch.cuda.graph(g, stream=cap):
        if mode == "serial":
            for j in (1, 2):
                pipe._ndt(j)
                outs.append(pipe._fwd(j))
        elif mode == "subgraph":
            for j in (1, 2):
                pipe.g_ndt[j].replay()
                pipe.g_fwd[j].replay()
                outs.append(pipe.out[j])
        else:
            s_ndt = pipe.s_ndts[0]
            ev[0].record(cap)
            s_ndt.wait_event(ev[0])
            for s in pipe.s_fwds:
                s.wait_event(ev[0])
            for i, j in enumerate((1, 2)):
                if mode == "fork":
                    pipe._ndt(j)  # on the capture stream
                    ev[1 + i].record(cap)
                else:
                    with torch.cuda.stream(s_ndt):
                        pipe._ndt(j)
                    ev[1 + i].record(s_ndt)
                s_f = pipe.s_fwds[j % F]
                s_f.wait_event(ev[1 + i])
                with torch.cuda.stream(s_f):
                    outs.append(pipe._fwd(j))
                ev[4 + i].record(s_f)
            # join every side stream back to the capture stream
            for i in range(2):
                if mode == "unjoined" and i == 1:
                    continue
                cap.wait_event(ev[4 + i])
            if mode != "fork":
                ev[7].record(s_ndt)
                cap.wait_event(ev[7])
        print(f"[{mode}] ending capture", flush=True)
    print(f"[{mode}] captured", flush=True)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(outs, ref))
    print(f"[{mode}] replayed 3x; outputs equal the eager steps: {same}", flush=True)
    sys.exit(0 if same else 3)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    for mode in sys.argv[1:] or MODES:
        p = subprocess.run([sys.executable, "-u", __file__, "--child", mode], capture_output=True, text=True,
                           timeout=240)
        tail = (p.stdout + p.stderr).strip().splitlines()
        msg = [l for l in tail if l.startswith(f"[{mode}]") or "Error" in l or "error" in l or "Fatal" in l][-4:]
        print(f"{mode:9s} rc {p.returncode}: " + " | ".join(msg), flush=True)
        if p.returncode < 0 or p.returncode >= 128:  # a signal (segfault, abort): nothing more on the GPU
            print(f"stopping after {mode}: the child died by a signal", flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
