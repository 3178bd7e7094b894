"""The static inline-asm checks of tools/check_dpp_hazards.py (run on every
translation unit by mcp_amd/build.py and on every generated module), pinned on
real gfx950 ISA: the r01 build of the C4 kernel with its Schur formation
unrolled ×5, which returned wrong iterates on the GPU, must be rejected; the same
variant built from the fixed sources (broadcast in uniform control flow) must pass."""

from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "tools", "check_dpp_hazards.py")
ISA = os.path.join(ROOT, "tests", "golden", "isa")


def run(path):
    return subprocess.run([sys.executable, CHECK, path], capture_output=True, text=True)


def test_rejects_the_wrong_iterate_build():
    """tests/golden/isa/c4_schur_unroll5_r01.s: excerpt of mcpx_nl_solve_schur (lane
    change, T = 2) with `#pragma unroll 5` on the Schur k-loop, r01 sources: inside
    `if (remaining row) eliminate_row(...)` (s_and_saveexec_b64) the allocator
    reloads 18 of the broadcast's 30 source VGPRs from AGPRs, for the active lanes
    only; the asm then reads the (inactive) pivot lane's stale registers."""
    r = run(os.path.join(ISA, "c4_schur_unroll5_r01.s"))
    assert r.returncode == 1
    assert "NARROWED-EXEC BROADCAST" in r.stdout and "18 of its 30 source VGPRs redefined" in r.stdout


def test_accepts_the_fixed_build():
    """Same kernel and unroll from the fixed sources: the reloads still happen
    (AGPR pressure is unchanged), but at full EXEC before the broadcast."""
    path = os.path.join(ISA, "c4_schur_unroll5_fixed.s")
    assert "v_accvgpr_read" in open(path).read()
    r = run(path)
    assert r.returncode == 0, r.stdout
    assert "0 narrowed-EXEC broadcasts" in r.stdout


def _write(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text("\t.text\nkern_mcpx:\n" + body)
    return str(p)


def test_dpp_wait_states(tmp_path):
    bad = _write(tmp_path, "\tv_mov_b32 v2, v7\n;;#ASMSTART\n\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] row_newbcast:1\n;;#ASMEND\n")
    assert run(bad).returncode == 1
    ok = _write(tmp_path, "\tv_mov_b32 v2, v7\n;;#ASMSTART\n\ts_nop 1\n\tv_fmac_f64_dpp v[4:5], v[2:3], v[6:7] row_newbcast:1\n;;#ASMEND\n")
    assert run(ok).returncode == 0


def test_exec_restore_ends_the_region(tmp_path):
    body = ("\ts_and_saveexec_b64 s[0:1], vcc\n\tv_mov_b32 v3, 0\n\ts_or_b64 exec, exec, s[0:1]\n\tv_mov_b32 v2, v9\n"
            ";;#ASMSTART\n\ts_mov_b64 s[4:5], exec\n\ts_mov_b64 exec, s[6:7]\n\tv_readfirstlane_b32 s8, v2\n"
            "\ts_mov_b64 exec, s[4:5]\n\ts_nop 1\n;;#ASMEND\n")
    assert run(_write(tmp_path, body)).returncode == 0
    body_bad = body.replace("\ts_or_b64 exec, exec, s[0:1]\n", "")
    r = run(_write(tmp_path, body_bad))
    assert r.returncode == 1 and "1 of its 1 source VGPRs redefined" in r.stdout
