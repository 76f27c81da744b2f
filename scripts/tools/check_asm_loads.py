#!/usr/bin/env python3
"""Audit inline-asm loads in a built code object (the pipelined paged decode issues its
K/V loads as inline asm with hand-counted waits).

hipcc does not know an asm load is still in flight: its VGPR destination counts as written at
`;;#ASMEND` (cdna_hip_programming.md §5.7 item 1), so a compiler `v_mov` / spill / reuse of those
registers before the matching `s_waitcnt vmcnt` reads stale data without any fault.  This walks
the device assembly of every kernel: for each asm `global_load_* ... nt` it follows program
order until a `s_waitcnt vmcnt(N)` retires the load (N <= the number of vector-memory ops
issued after it), and reports any instruction in between that reads or writes the load's
destination registers (see ``_walk`` for which paths).

    python scripts/tools/check_asm_loads.py lumen/csrc/kernels/paged_attention.hip [--kernel pa_]
Exit status 1 when a hazard is found.  tests/test_asm_loads_cpu.py runs it on the paged decode:
the pipelined kernel is dispatched only for the head sizes / GQA groups it passes (D = 128, or
one query head per KV head); the others spill asm results (D = 32, G = 8: a
``v_accvgpr_write`` of the destination right after the issue) and take the compiler-visible
variant."""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

VMEM = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)(load|store|atomic)")
WAIT = re.compile(r"s_waitcnt\b.*vmcnt\((\d+)\)")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
LABEL = re.compile(r"^(\.LBB[\w]+):")


def regs(text: str):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def functions(asm: str):
    """{kernel symbol: [instruction lines]} from hipcc -S output."""
    out, cur, name = {}, None, None
    for line in asm.splitlines():
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not line.startswith(".") and "@" in (m.group(2) or ""):
            name, cur = m.group(1), []
            out[name] = cur
            continue
        if cur is not None:
            if "s_endpgm" in line:
                cur.append(line)
                cur = None
                continue
            cur.append(line)
    return out


UBR = re.compile(r"^\s*s_branch\s+(\.LBB\w+)")
CBR = re.compile(r"^\s*s_cbranch_\w+\s+(\.LBB\w+)")


def _walk(lines, labels, i, dst, all_paths=False, max_states=20000, cap=32):
    """Follow the asm load at ``i`` until a ``s_waitcnt vmcnt`` retires it; the first line in
    between that reads or writes its destination registers, or None.

    Default: the straight-line region after the issue -- conditional branches fall through, the
    walk ends at an unconditional branch.  That is where hipcc puts the copy / spill / rematerial-
    isation of an asm result it believes is ready (it does so right at the definition), and the
    form that needs no path feasibility: the loop protocol around it (a wait of the older set
    before every use, ``vmcnt(0)`` before every ``break``) is reviewed in the source.
    ``all_paths`` explores both ways of every branch and every back-edge -- it also walks paths
    the loop's induction makes infeasible (a set consumed after an exit that never issued it),
    so its reports need reading by hand."""
    stack, seen = [(i + 1, 0)], set()
    while stack and len(seen) < max_states:
        j, younger = stack.pop()
        while j < len(lines):
            key = (j, min(younger, cap))
            if key in seen:
                break
            seen.add(key)
            s = lines[j].split(";")[0]
            st = s.strip()
            w = WAIT.search(s)
            if w and younger >= int(w.group(1)):
                break  # retired on this path
            if "s_endpgm" in st or st.startswith("s_setpc"):
                break
            if VMEM.match(s):
                younger += 1
            elif st and not w and not LABEL.match(lines[j]) and not st.startswith((".", "s_")):
                if regs(s) & dst:
                    return j
            u = UBR.match(s)
            if u:
                if not all_paths or u.group(1) not in labels:
                    break
                j = labels[u.group(1)] + 1
                continue
            c = CBR.match(s)
            if c and all_paths and c.group(1) in labels:
                stack.append((labels[c.group(1)] + 1, younger))
            j += 1
    return None


def audit(lines, all_paths: bool = False):
    """(asm nt loads, hazards) of one kernel body; a hazard is (load line, touching line,
    load text, touching text)."""
    labels = {}
    for i, l in enumerate(lines):
        m = LABEL.match(l)
        if m:
            labels[m.group(1)] = i
    hazards, n_loads = [], 0
    in_asm = False
    for i, l in enumerate(lines):
        if ";;#ASMSTART" in l:
            in_asm = True
            continue
        if ";;#ASMEND" in l:
            in_asm = False
            continue
        if not (in_asm and VMEM.match(l) and " nt" in l and "load" in l):
            continue
        n_loads += 1
        j = _walk(lines, labels, i, regs(l.split(",")[0]), all_paths)
        if j is not None:
            hazards.append((i, j, lines[i].strip(), lines[j].strip()))
    return n_loads, hazards


def device_asm(source: str, arch: str = "gfx950") -> str:
    inc = os.path.dirname(os.path.abspath(source))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", f"--offload-arch={arch}", "-O3", "-std=c++17",
                        "-munsafe-fp-atomics", "--cuda-device-only", "-S", f"-I{inc}", source,
                        "-o", out], check=True, capture_output=True)
        with open(out) as f:
            return f.read()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--kernel", default="", help="only kernels whose symbol contains this")
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("--all-paths", action="store_true",
                    help="explore both ways of every branch (reports infeasible paths too)")
    ap.add_argument("--asm", default="", help="audit this hipcc -S output instead of compiling")
    a = ap.parse_args(argv)
    asm = open(a.asm).read() if a.asm else device_asm(a.source, a.arch)
    total, bad = 0, 0
    for name, lines in functions(asm).items():
        if a.kernel and a.kernel not in name:
            continue
        n, hz = audit(lines, all_paths=a.all_paths)
        if n:
            print(f"{name[:90]}: {n} asm nt loads, {len(hz)} hazards")
        total += n
        for (i, j, ld, use) in hz[:5]:
            print(f"   load   [{i}] {ld}\n   touched [{j}] {use}")
        bad += len(hz)
    print(f"total asm nt loads {total}, hazards {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
