"""Static checks of the built gfx950 code objects (no GPU needed).

ADVICE r4 (medium): k_welford_q's heavy-ND loop issues its LDS reads as
inline asm (hv_issue) and orders their use by one later `s_waitcnt` asm
(hv_wait).  The compiler does not know those registers are still being
loaded, so a copy, spill or move of one between the two would read stale
data without any test noticing.  These tests read the code objects inside
lib/libndnet_amd.so (its .hip_fatbin section) and check that

* k_welford_q has no scratch and no VGPR spills (a spill could move a
  register the hardware is still writing), and
* in k_welford_q's machine code no instruction reads or writes the
  destination registers of an LDS load before an `s_waitcnt lgkmcnt(N)` that
  retires that load (LDS operations complete in order, so lgkmcnt(N) retires
  all but the newest N of them) -- the property the inline asm relies on.
"""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ndt-net_amd", "lib", "libndnet_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


def _code_objects(tmp_path):
    """The gfx950 code objects of every bundle in the library's .hip_fatbin."""
    objcopy = _tool("llvm-objcopy")
    if not objcopy or not os.path.exists(LIB):
        pytest.skip("llvm-objcopy or the built library is missing")
    fb = tmp_path / "fatbin.bin"
    subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fb}", LIB, str(tmp_path / "lib.so")], check=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for s in starts:  # bundle: magic, u64 entries, then (u64 offset, u64 size, u64 id size, id) per entry
        n = struct.unpack_from("<Q", data, s + len(MAGIC))[0]
        p = s + len(MAGIC) + 8
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            tid = data[p + 24:p + 24 + idlen].decode()
            p += 24 + idlen
            if "gfx950" in tid and size:
                path = tmp_path / f"co_{len(out)}.elf"
                path.write_bytes(data[s + off:s + off + size])
                out.append(path)
    assert out, "no gfx950 code object in the library"
    return out


def _kernel_meta(cos):
    readelf = _tool("llvm-readelf")
    if not readelf:
        pytest.skip("llvm-readelf is missing")
    meta = {}
    for co in cos:
        txt = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
        cur = None
        for line in txt.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                cur = meta.setdefault(m.group(1), {})
                continue
            m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count|vgpr_count):\s+(\d+)",
                         line)
            if m and cur is not None:
                cur[m.group(1)] = int(m.group(2))
    return meta


def test_welford_kernels_have_no_scratch_or_spills(tmp_path):
    meta = _kernel_meta(_code_objects(tmp_path))
    wq = {k: v for k, v in meta.items() if "k_welford_q" in k}
    assert len(wq) == 4, sorted(meta)  # float and double inputs x the two light forms
    for name, m in wq.items():
        assert m["private_segment_fixed_size"] == 0, (name, m)
        # (SGPR spills go to VGPR lanes, v_writelane / v_readlane: no memory, and
        # they never copy a VGPR an LDS load is writing)
        assert m["vgpr_spill_count"] == 0, (name, m)


_REG = re.compile(r"\b([vas])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def _regs(text):
    regs = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        lo, hi = (int(m.group(2)), int(m.group(3))) if m.group(2) else (int(m.group(4)), int(m.group(4)))
        regs.update((kind, r) for r in range(lo, hi + 1))
    return regs


def _lds_hazards(lines):
    """(address, instruction) pairs that touch an LDS load's destination
    before an lgkmcnt wait retires it (straight-line scan; state cleared at
    branch targets, where the compiler's own waits govern)."""
    insns = []
    for ln in lines:
        m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):", ln)
        if m:
            insns.append((int(m.group(2), 16), m.group(1)))
    targets = set()
    for addr, ins in insns:  # SOPP branches: target = pc + 4 + 4 * simm16
        m = re.match(r"s_c?branch\S*\s+(\d+)", ins)
        if m:
            imm = int(m.group(1))
            targets.add(addr + 4 + 4 * (imm - 65536 if imm >= 32768 else imm))
    pending = []  # FIFO of outstanding LDS ops: set of destination registers (empty for stores)
    bad = []
    for addr, ins in insns:
        if addr in targets:
            pending = []
        op = ins.split()[0]
        if op == "s_waitcnt" or op.startswith("s_waitcnt_lgkmcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", ins)
            if m:
                keep = int(m.group(1))
                pending = pending[len(pending) - keep:] if keep < len(pending) else pending
                if keep == 0:
                    pending = []
            continue
        live = set().union(*pending) if pending else set()
        if op.startswith("ds_"):
            args = ins[len(op):].split(",")
            returns = op.startswith(("ds_read", "ds_load", "ds_bpermute", "ds_permute", "ds_swizzle")) or "_rtn" in op
            dst = _regs(args[0]) if returns else set()
            srcs = _regs(",".join(args[1:] if returns else args))
            if live & (srcs | dst):
                bad.append((hex(addr), ins))
            pending.append(dst)
            continue
        if live & _regs(ins[len(op):]):
            bad.append((hex(addr), ins))
    return bad


def test_welford_lds_loads_are_not_touched_before_their_wait(tmp_path):
    objdump = _tool("llvm-objdump")
    if not objdump:
        pytest.skip("llvm-objdump is missing")
    checked = 0
    for co in _code_objects(tmp_path):
        txt = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(co)], check=True, capture_output=True,
                             text=True).stdout
        for block in re.split(r"\n(?=[0-9a-f]+ <)", txt):
            head = block.split("\n", 1)[0]
            if "k_welford_q" not in head:
                continue
            lines = block.split("\n")[1:]
            n_ds = sum(1 for ln in lines if "ds_read_b128" in ln)
            assert n_ds > 0, head
            hz = _lds_hazards(lines)
            assert not hz, f"{head}: registers of an outstanding LDS load touched: {hz[:5]}"
            checked += 1
    assert checked == 4


def test_hazard_scan_flags_an_early_use():
    """The scan itself: a use of a loaded register before its wait is flagged,
    after lgkmcnt(N) only the newest N loads stay outstanding."""
    mk = lambda i, s: f"\t{s} // {0x100 + 4 * i:012X}: 00000000"  # noqa: E731
    prog = ["ds_read_b128 v[4:7], v1 offset:64", "ds_read_b128 v[8:11], v1 offset:80",
            "s_waitcnt lgkmcnt(1)", "v_mov_b32_e32 v2, v4", "v_mov_b32_e32 v3, v9"]
    bad = _lds_hazards([mk(i, s) for i, s in enumerate(prog)])
    assert [b[1] for b in bad] == ["v_mov_b32_e32 v3, v9"]
    assert not _lds_hazards([mk(i, s) for i, s in enumerate(prog[:3] + ["s_waitcnt lgkmcnt(0)"] + prog[3:])])
