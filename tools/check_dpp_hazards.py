"""Static check of VALU-write → cross-lane-read hazards around the inline asm.

A DPP instruction reading a VGPR that a VALU instruction wrote fewer than 2 wait
states earlier reads a stale value (gfx9 hazard table; hipcc does not pad
hazards whose consumer sits inside an asm statement).  Scans the .s of a
-save-temps build: for every *_dpp instruction, walks back through the
preceding instructions counting wait states (an instruction = 1, s_nop N = N+1)
and flags a VALU write to the DPP source register (src0) within 2 states.

    python tools/check_dpp_hazards.py path/to/file.s [kernel-substring]
"""

from __future__ import annotations

import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(tok: str) -> set:
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().split("\n")
    kernel = None
    insts = []  # (kernel, text, in_asm)
    in_asm = False
    for l in lines:
        if ";;#ASMSTART" in l:
            in_asm = True
        if ";;#ASMEND" in l:
            in_asm = False
        t = l.split(";")[0].strip()
        if t.endswith(":") and not t.startswith(".") and "_Z" in t:
            kernel = t[:-1]
            continue
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        insts.append((kernel, t, in_asm))
    bad = 0
    checked = 0
    for i, (k, t, asm) in enumerate(insts):
        op = t.split()[0]
        if want and want not in (k or ""):
            continue
        ops = [x.strip() for x in t[len(op):].split(",")]
        if "_dpp" in op and len(ops) >= 2:
            src, need = regs(ops[1]), 2          # VALU write → DPP read: 2 wait states
        elif asm and (op.startswith("v_readfirstlane") or op.startswith("v_readlane")) and len(ops) >= 2:
            src, need = regs(ops[1]), 1          # VALU write → v_readlane/readfirstlane: 1
        elif asm and op.startswith("v_permlane") and len(ops) >= 2:
            src, need = regs(ops[0]) | regs(ops[1]), 2
        else:
            continue
        checked += 1
        states = 0
        j = i - 1
        while j >= 0 and states < need:
            kk, tt, _ = insts[j]
            if kk != k:
                break
            o = tt.split()[0]
            if o == "s_nop":
                states += int(tt.split()[1], 0) + 1
                j -= 1
                continue
            if o.startswith("v_") and not o.startswith("v_readfirstlane") and not o.startswith("v_readlane") \
                    and not o.startswith("v_cmp"):
                dst = regs(tt[len(o):].split(",")[0])
                if dst & src:
                    bad += 1
                    print(f"HAZARD in {k}:\n   {tt}\n   {t}  ({states} wait states between)")
            states += 1
            j -= 1
    print(f"checked {checked} DPP / asm cross-lane instructions, {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
