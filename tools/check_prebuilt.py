"""Before a GPU call: is the tree built?  libmcpx.so from the current sources, and every generated
module the GPU tests, smoke() and bench.py load present in mcp_amd/_gen under its current key —
a missing one would be compiled on the GPU box (minutes of hipcc with no output).  CPU only.

    python tools/check_prebuilt.py      (exit 1 and the missing pieces otherwise)
"""

from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    from mcp_amd import build as B

    bad = []
    if B._stale():
        bad.append("mcp_amd/libmcpx.so is not built from the current sources")
    from mcp_amd.lane_change import LaneChangeGame
    from tests.test_nonlinear import cubic_mcp, trig_mcp
    from tests.test_sensitivity_nl import poly_mcp

    nls = [LaneChangeGame(T).mcp.nl for T in (2, 10)] + [m.nl for m in (cubic_mcp(), trig_mcp(), poly_mcp(40, 30))]
    for nl in nls:
        p = nl.module_path()
        if not os.path.exists(p):
            bad.append(f"missing module {os.path.relpath(p, ROOT)} (n={nl.n}, m={nl.m})")
    for b in bad:
        print(b)
    print("prebuilt: ok" if not bad else f"prebuilt: {len(bad)} missing")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
