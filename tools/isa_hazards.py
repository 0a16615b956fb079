#!/usr/bin/env python3
"""Scan gfx950 machine code for the VMEM store-data hazard.

A vector-memory store with more than 64 bits of data (buffer/global/flat *_dwordx3 / x4, b96 /
b128) reads its data VGPRs after it issues. A VALU instruction that overwrites one of them within
2 wait states of the store can change what the store writes -- on gfx950 this was observed for
buffer stores with an SGPR `soffset`, for which LLVM's hazard recognizer inserts no wait states
(it exempts MUBUF stores whose soffset is a register). The failure is timing-dependent: only
some lanes of component 0 were corrupted, and which rows varied from run to run.

Usage:
    python tools/isa_hazards.py LIB.so|FILE.s [...]    -> prints violations, exit 1 if any

Input: a shared library / object with embedded clang offload bundles (the gfx950 code objects
are extracted and disassembled with llvm-objdump), or a `hipcc -S --cuda-device-only` .s file.
"""
from __future__ import annotations

import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NEED = 2  # wait states a VALU write of store data must keep from a >64-bit store (gfx940+)

_WIDE_STORE = re.compile(r"^(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\b")
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def code_objects(blob: bytes):
    """Yield (triple, elf bytes) of every entry of every offload bundle in blob."""
    pos = 0
    while True:
        i = blob.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", blob, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if size:
                yield triple, blob[i + off:i + off + size]
        pos = i + len(MAGIC)


def disassemble(path: Path) -> list[str]:
    if path.suffix == ".s":
        return path.read_text().splitlines()
    lines: list[str] = []
    blob = path.read_bytes()
    with tempfile.TemporaryDirectory() as td:
        for k, (triple, elf) in enumerate(code_objects(blob)):
            if "gfx950" not in triple:
                continue
            f = Path(td) / f"co{k}.elf"
            f.write_bytes(elf)
            out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(f)], capture_output=True,
                                 text=True, check=True).stdout
            lines += out.splitlines()
    return lines


def _regs(tok: str) -> set[int]:
    m = _VREG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def parse(lines: list[str]):
    """-> list of (mnemonic, operand tokens, text, function name, address or None); labels /
    directives dropped. The address is objdump's `// 0000ADDR:` comment (absent in .s files)."""
    insts = []
    fn = "?"
    for raw in lines:
        am = re.search(r"//\s*([0-9A-Fa-f]{8,}):", raw)
        addr = int(am.group(1), 16) if am else None
        s = raw.split("//")[0].split(";")[0].rstrip()
        if not s:
            continue
        m = re.match(r"^(?:[0-9a-f]+\s+)?<([^>]+)>:$", s.strip())  # objdump function header
        if m:
            fn = m.group(1)
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:", s):  # .s label (function or block)
            if not s.startswith((".L", "$")):
                fn = s.split(":")[0]
            insts.append(("<label>", [s.split(":")[0]], s, fn, None))
            continue
        st = s.strip()
        if st.startswith("."):
            continue
        parts = st.split(None, 1)
        mn = parts[0]
        if not re.match(r"^[a-z][a-z0-9_]*$", mn):
            continue
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        insts.append((mn, ops, st, fn, addr))
    return insts


def wait_states(mn: str, ops: list[str]) -> int:
    if mn == "s_nop":
        try:
            return int(ops[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def _branch_target(insts, j, by_addr, by_label):
    """Index of the instruction a branch at j jumps to, or None when it cannot be resolved."""
    mn, ops, _, _, addr = insts[j]
    if not ops:
        return None
    tok = ops[0]
    if tok in by_label:  # .s input: a label operand
        return by_label[tok]
    try:
        imm = int(tok, 0)
    except ValueError:
        return None
    if addr is None:
        return None
    off = imm - 0x10000 if imm >= 0x8000 else imm  # simm16, in dwords, from the next instruction
    return by_addr.get(addr + 4 + 4 * off)


def scan(insts, taken=False) -> list[str]:
    """Every path from a >64-bit store is followed for NEED wait states. Straight-line code and
    the fall-through of a conditional branch are always followed (a not-taken
    s_cbranch does not end the window). A path ends at s_branch, s_setpc or s_endpgm.

    taken=True also follows the target of every branch, counting the branch as one wait state
    (LLVM's own cross-block count: it pads a loop head after a store + back edge with s_nop 0).
    While EXEC is unchanged since the store, a taken s_cbranch_execz (or a not-taken
    s_cbranch_execnz) means the store ran with EXEC = 0 and wrote nothing: no hazard on that
    path. DESIGN.md 5.1b reports what the taken-branch scan finds and why the product does not
    assert it."""
    by_addr = {ins[4]: k for k, ins in enumerate(insts) if ins[4] is not None}
    by_label = {ins[1][0]: k for k, ins in enumerate(insts) if ins[0] == "<label>"}
    bad = []
    for i, (mn, ops, text, fn, _) in enumerate(insts):
        if not _WIDE_STORE.match(mn):
            continue
        # data operand: buffer stores "vdata, vaddr, srsrc, soffset"; global/flat "vaddr, vdata, ..."
        data = _regs(ops[0]) if mn.startswith("buffer") else _regs(ops[1] if len(ops) > 1 else "")
        if not data:
            continue
        work = [(i + 1, 0, False)]  # (index, wait states so far, EXEC written since the store)
        seen = set()
        hit = None
        while work and hit is None:
            j, ws, exw = work.pop()
            while j < len(insts) and ws < NEED and (j, ws, exw) not in seen:
                seen.add((j, ws, exw))
                mn2, ops2, text2, _, _ = insts[j]
                if mn2 == "<label>":
                    j += 1
                    continue
                if mn2.startswith("v_") and ops2 and _regs(ops2[0]) & data:
                    hit = f"{fn}: '{text}' then '{text2}' after {ws} wait state(s)"
                    break
                if mn2.startswith(("s_setpc", "s_endpgm")):
                    break
                if mn2.startswith(("s_branch", "s_cbranch")):
                    if taken:
                        t = _branch_target(insts, j, by_addr, by_label)
                        if t is None:
                            hit = f"{fn}: '{text}' then unresolved branch '{text2}'"
                            break
                        if not (mn2 == "s_cbranch_execz" and not exw):
                            work.append((t, ws + 1, exw))
                    if mn2.startswith("s_branch") or (mn2 == "s_cbranch_execnz" and not exw):
                        break
                if mn2.startswith("s_") and (("saveexec" in mn2) or (ops2 and ops2[0].startswith("exec"))):
                    exw = True
                ws += wait_states(mn2, ops2)
                j += 1
        if hit:
            bad.append(hit)
    return bad


def main(argv: list[str]) -> int:
    total = 0
    for a in argv:
        insts = parse(disassemble(Path(a)))
        stores = sum(1 for mn, *_ in insts if _WIDE_STORE.match(mn))
        bad = scan(insts)
        tk = [x for x in scan(insts, taken=True) if x not in bad]
        total += len(bad)
        print(f"{a}: {len(insts)} instructions, {stores} wide stores, {len(bad)} hazard(s) on "
              f"straight-line / fall-through paths, {len(tk)} more through a taken branch")
        for b in bad[:20]:
            print("  ", b)
        for b in tk[:20]:
            print("   (taken)", b)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
