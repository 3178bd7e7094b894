"""Static checks of the inline asm's cross-lane reads in a gfx950 .s (-save-temps).

1. Wait states.  A DPP instruction reading a VGPR that a VALU instruction wrote
   fewer than 2 wait states earlier reads a stale value (gfx9 hazard table);
   v_readlane / v_readfirstlane need 1, v_permlane*_swap 2, and a v_writelane
   whose lane-select SGPR a VALU wrote needs 4.  hipcc does not pad
   hazards whose consumer sits inside an asm statement.  For every such reader,
   walk back through the preceding instructions counting wait states (an
   instruction = 1, s_nop N = N+1) and flag a VALU write to its source.

2. EXEC-switched broadcasts under a compiler-narrowed EXEC.  The broadcast asm
   (csrc/bcast_group.inc) saves EXEC, sets it to the pivot lane and reads that
   lane's VGPRs with v_readfirstlane.  If the asm sits inside a divergent region
   (after s_and_saveexec_b64 & co. without the matching restore), the pivot lane
   is typically inactive there, and any copy the compiler places into the asm's
   input registers inside the region — a reload of a spilled value from an AGPR,
   a register move — skips that lane: the asm then broadcasts a stale value.
   This is how the ×5-unrolled C4 Schur formation returned wrong iterates
   (DESIGN.md §4).  The kernels broadcast in uniform control flow; every
   EXEC-switching asm block is walked back along its fall-through path to the
   nearest label / unconditional branch / EXEC restore, and an EXEC narrowing met
   first is a hazard (the number of source registers redefined in between is
   reported).

3. EXEC writes inside inline asm followed by a DPP instruction within 5 wait states (the
   gfx9 table's EXEC-write → DPP distance, applied conservatively to SALU writes too, which
   the compiler cannot pad for when they sit inside asm).

4. An MFMA result read by an inline-asm instruction too early.  A VALU, LDS, buffer/global
   or export instruction reading a VGPR that `v_mfma_f64_16x16x4_f64` wrote needs 19
   independent instructions in between (the dependency table of the CDNA3/4 ISA; LLVM's
   DMFMA16x16WriteVgprVALUReadWaitStates / …MemExpReadWaitStates; 6 after the 4x4x4 DGEMM,
   and 19 is taken for every other MFMA too).  hipcc pads this for its own instructions, not
   for a consumer inside an asm string: the round-4 Gauss-Jordan that recorded pivot 0 by a
   one-lane `ds_write_b64` of the accumulator right after the Schur MFMAs stored the register's
   stale value, and every C3 instance came back a few ulps off.  The walk
   stops at a label: the kernels' MFMA results are consumed in the block that computed them.

    python tools/check_dpp_hazards.py path/to/file.s [kernel-substring]
Exit status 1 if any hazard is found.
"""

from __future__ import annotations

import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")
SREG = re.compile(r"s\[(\d+):(\d+)\]|\bs(\d+)\b")
NARROW = ("s_and_saveexec_b64", "s_andn2_saveexec_b64", "s_and_saveexec_b32")
EXEC_WRITES = ("s_and_b64", "s_andn2_b64", "s_xor_b64", "s_or_b64", "s_mov_b64", "s_cselect_b64")


def regs(tok: str) -> set:
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(path: str):
    """[(kernel, text, in_asm, is_label)] in file order."""
    kernel = None
    out = []
    in_asm = False
    for l in open(path).read().split("\n"):
        if ";;#ASMSTART" in l:
            in_asm = True
        if ";;#ASMEND" in l:
            in_asm = False
        t = l.split(";")[0].strip()
        if t.endswith(":") and not t.startswith(".") and ("_Z" in t or "mcpx" in t):
            kernel = t[:-1]
            continue
        if t.endswith(":") and t.startswith(".LBB"):
            out.append((kernel, t, in_asm, True))
            continue
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        out.append((kernel, t, in_asm, False))
    return out


def sregs(tok: str) -> set:
    out = set()
    for m in SREG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def valu_sdst(t: str) -> set:
    """SGPRs a VALU instruction writes (v_readlane / v_readfirstlane / VOP3 compares)."""
    o = t.split()[0]
    if o.startswith("v_"):
        return sregs(t[len(o):].split(",")[0])
    return set()


def valu_dst(t: str) -> set:
    o = t.split()[0]
    if o.startswith("v_") and not o.startswith(("v_readfirstlane", "v_readlane", "v_cmp")):
        return regs(t[len(o):].split(",")[0])
    return set()


def exec_dpp_hazards(insts, want: str):
    """3. A DPP instruction fewer than 5 wait states after an EXEC write: an EXEC write inside
    inline asm before any DPP (the EXEC switch of a broadcast; the compiler cannot pad for the
    asm's), or any EXEC write — the compiler's restore after a divergent `if` included — before a
    DPP inside asm (the compiler pads its own DPP, not an asm one).  The band kernel's DPP
    variant (r05) lost lanes this way: `if (lane == p) {…}` ended with `s_or_b64 exec` two
    instructions before the asm `v_fmac_f64_dpp`, which then ran under the narrowed EXEC."""
    bad = []
    for i, (k, t, asm, lab) in enumerate(insts):
        if lab or "_dpp" not in t.split()[0] or (want and want not in (k or "")):
            continue
        states, j = 0, i - 1
        while j >= 0 and states < 5:
            kk, tt, a, ll = insts[j]
            if kk != k or ll:
                break
            o = tt.split()[0]
            if o == "s_nop":
                states += int(tt.split()[1], 0) + 1
                j -= 1
                continue
            if (a or asm) and re.match(r"s_\S+\s+exec\b", tt):
                bad.append(f"EXEC→DPP HAZARD in {k}:\n   {tt}\n   {t}  ({states} wait states between)")
                break
            states += 1
            j -= 1
    return bad


def wait_state_hazards(insts, want: str):
    bad, checked = [], 0
    for i, (k, t, asm, lab) in enumerate(insts):
        if lab or (want and want not in (k or "")):
            continue
        op = t.split()[0]
        ops = [x.strip() for x in t[len(op):].split(",")]
        if "_dpp" in op and len(ops) >= 2:
            src, need = regs(ops[1]), 2          # VALU write → DPP read: 2 wait states
        elif asm and (op.startswith("v_readfirstlane") or op.startswith("v_readlane")) and len(ops) >= 2:
            src, need = regs(ops[1]), 1          # VALU write → v_readlane/readfirstlane: 1
        elif asm and op.startswith("v_permlane") and len(ops) >= 2:
            src, need = regs(ops[0]) | regs(ops[1]), 2
        elif asm and op.startswith("v_writelane") and len(ops) >= 3:
            # lane select written by a VALU: 4 wait states (VGPR sources: none)
            checked += 1
            sel, states, j = sregs(ops[2]), 0, i - 1
            if not sel:  # inline-constant lane select: nothing to wait for
                continue
            while j >= 0 and states < 4:
                kk, tt, _, ll = insts[j]
                if kk != k or ll:
                    if ll:
                        bad.append(f"WAIT-STATE HAZARD (join point {tt}) in {k}:\n   {t}")
                    break
                if tt.split()[0] == "s_nop":
                    states += int(tt.split()[1], 0) + 1
                elif valu_sdst(tt) & sel:
                    bad.append(f"WAIT-STATE HAZARD in {k}:\n   {tt}\n   {t}  ({states} wait states between)")
                    states += 1
                else:
                    states += 1
                j -= 1
            continue
        else:
            continue
        checked += 1
        states = 0
        j = i - 1
        while j >= 0 and states < need:
            kk, tt, _, ll = insts[j]
            if kk != k:
                break
            if ll:
                # a join point: another predecessor (a branch to this label) may have
                # written the source just before jumping; only the fall-through path
                # is walked, so an asm reader this close to a label is reported unless
                # it is padded on its own.  A compiler-emitted DPP (a builtin, outside
                # asm) is padded by the compiler's hazard recognizer, which follows
                # every predecessor block.
                if asm:
                    bad.append(f"WAIT-STATE HAZARD (join point {tt}) in {k}:\n   {t}  ({states} wait states after the label)")
                break
            o = tt.split()[0]
            if o == "s_nop":
                states += int(tt.split()[1], 0) + 1
                j -= 1
                continue
            if valu_dst(tt) & src:
                bad.append(f"WAIT-STATE HAZARD in {k}:\n   {tt}\n   {t}  ({states} wait states between)")
            states += 1
            j -= 1
    return bad, checked


MFMA_READ_STATES = {"v_mfma_f64_16x16x4": 19, "v_mfma_f64_4x4x4": 6}


def mfma_need(op: str) -> int:
    for k, v in MFMA_READ_STATES.items():
        if op.startswith(k):
            return v
    return 19


def asm_vgpr_reads(t: str) -> set:
    """VGPRs an instruction reads: every operand of a store / DS write / export; the sources of a
    VALU op (and its destination for the accumulating / partial writers)."""
    op = t.split()[0]
    ops = [x.strip() for x in t[len(op):].split(",")]
    if op.startswith(("ds_write", "ds_store", "buffer_store", "global_store", "flat_store", "exp")):
        return set().union(*(regs(x) for x in ops)) if ops else set()
    if op.startswith(("ds_", "buffer_", "global_", "flat_")):  # loads: address operands only
        return set().union(*(regs(x) for x in ops[1:])) if len(ops) > 1 else set()
    if op.startswith("v_"):
        rd = set().union(*(regs(x) for x in ops[1:])) if len(ops) > 1 else set()
        if "fmac" in op or "_mac_" in op or op.startswith(("v_writelane", "v_permlane")):
            rd |= regs(ops[0])
        return rd
    return set()


def mfma_read_hazards(insts, want: str):
    """4. An asm instruction reading an MFMA's destination VGPRs fewer than mfma_need() wait
    states after the MFMA (same block)."""
    bad, checked = [], 0
    for i, (k, t, asm, lab) in enumerate(insts):
        if not asm or lab or (want and want not in (k or "")):
            continue
        live = asm_vgpr_reads(t)
        if not live:
            continue
        checked += 1
        states, j = 0, i - 1
        while j >= 0 and live and states < 19:
            kk, tt, _, ll = insts[j]
            if kk != k or ll:
                break
            o = tt.split()[0]
            if o == "s_nop":
                states += int(tt.split()[1], 0) + 1
                j -= 1
                continue
            if o.startswith("v_mfma"):
                hit = regs(tt[len(o):].split(",")[0]) & live
                if hit and states < mfma_need(o):
                    bad.append(f"MFMA-RESULT HAZARD in {k}:\n   {tt}\n   {t}  ({states} wait states between, "
                               f"{mfma_need(o)} needed)")
                    break
                live -= hit
            else:
                live -= valu_dst(tt)
            states += 1
            j -= 1
    return bad, checked


def exec_switch_blocks(insts):
    """Start indices of asm blocks that save EXEC and set it (s_mov_b64 sX, exec;
    s_mov_b64 exec, sY), with the VGPRs their v_readfirstlane read."""
    for i, (k, t, asm, lab) in enumerate(insts):
        if not asm or lab or i + 1 >= len(insts):
            continue
        if re.fullmatch(r"s_mov_b64\s+s\[\d+:\d+\],\s*exec", t) and insts[i + 1][1].startswith("s_mov_b64 exec"):
            src, j = set(), i + 2
            while j < len(insts) and insts[j][2] and not insts[j][1].startswith("s_mov_b64 exec"):
                if insts[j][1].startswith("v_readfirstlane"):
                    src |= regs(insts[j][1].split(",", 1)[1])
                j += 1
            yield i, src


def narrowed_exec_hazards(insts, want: str):
    bad, checked = [], 0
    for i, src in exec_switch_blocks(insts):
        k = insts[i][0]
        if want and want not in (k or ""):
            continue
        checked += 1
        redefined = set()
        j = i - 1
        while j >= 0:
            kk, tt, asm, lab = insts[j]
            if kk != k or lab:
                break  # a join point / another function: not this path's business
            o = tt.split()[0]
            if not asm:
                if o in ("s_branch", "s_setpc_b64", "s_endpgm"):
                    break  # not a fall-through predecessor
                wm = re.fullmatch(r"s_mov_b64\s+exec,\s*(s\[\d+:\d+\])", tt)
                if wm:  # the restore of a whole-wave-mode region (SGPR spills to VGPR lanes):
                    # `s_or_saveexec_b64 sX, -1` … `s_mov_b64 exec, sX` leaves EXEC as it was
                    w = j - 1
                    while w >= 0 and insts[w][0] == k and not insts[w][3]:
                        if re.search(r"\bexec\b", insts[w][1].split(",", 1)[0]) or insts[w][1].startswith("s_or_saveexec"):
                            break
                        w -= 1
                    if (w >= 0 and insts[w][0] == k and not insts[w][3]
                            and re.fullmatch(r"s_or_saveexec_b64\s+" + re.escape(wm.group(1)) + r",\s*-1", insts[w][1])):
                        j = w - 1
                        continue
                if o in NARROW or (o in EXEC_WRITES and re.match(r"\S+\s+exec,", tt) and o != "s_or_b64"
                                   and not (o == "s_mov_b64" and "exec, -1" in tt)):
                    bad.append(f"NARROWED-EXEC BROADCAST in {k}: the asm block at instruction {i} switches EXEC "
                               f"inside a divergent region opened by `{tt}`; {len(redefined & src)} of its "
                               f"{len(src)} source VGPRs redefined in between")
                    break
                if o == "s_or_b64" and re.match(r"s_or_b64\s+exec,", tt) or (o == "s_mov_b64" and "exec, -1" in tt):
                    break  # EXEC restored on this path
                if o.startswith("s_or_saveexec"):
                    break
            redefined |= valu_dst(tt)
            j -= 1
    return bad, checked


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    path = argv[0]
    want = argv[1] if len(argv) > 1 else ""
    insts = parse(path)
    w, wc = wait_state_hazards(insts, want)
    w += exec_dpp_hazards(insts, want)
    mf, mc = mfma_read_hazards(insts, want)
    w += mf
    wc += mc
    x, xc = narrowed_exec_hazards(insts, want)
    for msg in (w + x)[:50]:
        print(msg)
    print(f"checked {wc} DPP / asm cross-lane instructions and {xc} EXEC-switched broadcasts: "
          f"{len(w)} wait-state hazards, {len(x)} narrowed-EXEC broadcasts")
    return 1 if (w or x) else 0


if __name__ == "__main__":
    sys.exit(main())
