"""The kernel mask of a generated module is decided twice: by the C macros of
csrc/ipm_nl_kernel.hpp (MCPX_NL_CAN_*, compiled into mcpx_nl_meta — what the C ABI
launches) and by mcp_amd/codegen.py NLSystem.solvers() / wg_solvers() (what the oracle's
`wave_schur` mode and the front end assume).  A disagreement makes the GPU run the one-wave
Gauss-Jordan while the oracle runs the LU, so this test evaluates the C macros
with gcc at sizes around every limit and compares them with the Python formulas."""

from __future__ import annotations

import os
import re
import subprocess

import pytest

from mcp_amd import codegen

HDR = os.path.join(os.path.dirname(codegen.__file__), "csrc", "ipm_nl_kernel.hpp")
MACROS = ("MCPX_NL_CAN_REDUCED", "MCPX_NL_CAN_DENSE", "MCPX_NL_CAN_SCHUR", "MCPX_NL_CAN_WG_REDUCED",
          "MCPX_NL_CAN_WG_DENSE", "MCPX_NL_CAN_WG_SCHUR")


def _defines() -> str:
    """Every `#define MCPX_NL_…` of the header that the masks depend on (with continuations)."""
    text = open(HDR).read().replace("\\\n", " ")
    keep = []
    for line in text.splitlines():
        mt = re.match(r"\s*#define\s+(MCPX_NL_(?:CAN_\w+|SCHUR_LDS|NV|WG_LDS|WG_LIMIT|BAND_\w+))\b", line)
        if mt:
            keep.append(line.strip())
    return "\n".join(keep)


def _cases():
    out = []
    for n in (1, 16, 40, 47, 48, 63, 64, 65, 100, 200):
        for m in (0, 1, 50, 100, 127, 128, 129, 250):
            for has_s in (0, 1):
                out.append((n, m, has_s))
    return out


def _python_mask(n, m, has_s):
    nl = object.__new__(codegen.NLSystem)
    nl.n, nl.m, nl.has_s = n, m, bool(has_s)
    nl.OFF_S = n * n + 2 * n * m + n + m
    s, w = nl.solvers(), nl.wg_solvers()
    return (int(s["reduced"]), int(s["dense"]), int(s["schur"]), int(w["reduced"]), int(w["dense"]), int(w["schur"]))


def test_python_solver_masks_match_the_compiled_macros(tmp_path):
    cases = _cases()
    src = ["#include <stdio.h>", "int main(void) {"]
    for n, m, hs in cases:
        src += ["#undef MCPX_NL_N", "#undef MCPX_NL_M", "#undef MCPX_NL_HAS_S", f"#define MCPX_NL_N {n}",
                f"#define MCPX_NL_M {m}", f"#define MCPX_NL_HAS_S {hs}",
                '  printf("' + " ".join(["%d"] * len(MACROS)) + '\\n", ' + ", ".join(f"(int)({x})" for x in MACROS) + ");"]
    src += ["  return 0;", "}"]
    c = tmp_path / "masks.c"
    c.write_text(_defines() + "\n" + "\n".join(src) + "\n")
    exe = tmp_path / "masks"
    subprocess.run(["gcc", "-O0", "-o", str(exe), str(c)], check=True)
    rows = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for (n, m, hs), row in zip(cases, rows):
        got = tuple(int(v) for v in row.split())
        assert got == _python_mask(n, m, hs), (n, m, hs, got, _python_mask(n, m, hs))


@pytest.mark.parametrize("n,m", [(48, 128), (40, 50), (64, 128)])
def test_schur_lds_formula_is_the_macro(n, m):
    """The case ADVICE r04 named: n = 48, m = 128 fits the C limit; the Python formula agreed
    only after schur_lds_bytes took the n×(n+1) rows of [S | rr]."""
    nl = object.__new__(codegen.NLSystem)
    nl.n, nl.m, nl.has_s = n, m, False
    nl.OFF_S = n * n + 2 * n * m + n + m
    assert nl.schur_lds_bytes() == 8 * (n * n + 2 * n * m + n + m + n * (n + 1) + 3 * (n + 2 * m) + 4 * m)
