"""Variant builds of libmcpx.so for kernel A/B runs (tools/ab_c3.py, tools/c3_batch_curve.py
with MCPX_LIB_PATH): the translation units named by --tu get extra -D flags, every other
unit is the cached object of the product build (mcp_amd/build.py OBJ_CACHE).

    python tools/ab_build.py --name bperm --tu ipm_inst_spec.hip -D MCPX_GJ_BPERM=1
    -> tools/ablib/libmcpx_bperm.so

The variant is NOT hazard-checked (tools/check_dpp_hazards.py runs only in the product
build); run it through the checker before a GPU run when the variant touches inline asm.
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mcp_amd import build as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", required=True)
    ap.add_argument("--tu", action="append", required=True, help="translation unit (basename) built with the flags")
    ap.add_argument("-D", dest="defs", action="append", default=[])
    ap.add_argument("--allow-hazard", action="store_true",
                    help="build even if the checker flags the variant (reproducing a known hazard on purpose)")
    a = ap.parse_args()
    B.build(verbose=False)  # the product objects in the cache
    out_dir = os.path.join(ROOT, "tools", "ablib")
    os.makedirs(out_dir, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="mcpx_ab_")
    objs, procs = [], []
    flags = [f"-D{d}" for d in a.defs]
    for src in B.SOURCES:
        base = os.path.basename(src)
        obj = os.path.join(tmp, base + ".o")
        if base in a.tu:
            cmd = [B.HIPCC, *B.FLAGS, *flags, "-save-temps=obj", "-c", src, "-o", obj]
            procs.append(subprocess.Popen(cmd, cwd=tmp))
        else:
            cdir = os.path.join(B.OBJ_CACHE, base + "." + B._tu_key(src, B.FLAGS))
            shutil.copy2(os.path.join(cdir, base + ".o"), obj)
        objs.append(obj)
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("hipcc failed")
    for base in a.tu:  # the hazard check of the variant's device code
        stem = os.path.splitext(base)[0]
        asm = os.path.join(tmp, f"{stem}-hip-amdgcn-amd-amdhsa-gfx950.s")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_dpp_hazards.py"), asm],
                           capture_output=True, text=True)
        print(f"{base}: {r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]}")
        if r.returncode != 0:
            if not a.allow_hazard:
                raise SystemExit(f"hazard in {asm}")
            print("\n".join(r.stdout.splitlines()[:6]))
    lib = os.path.join(out_dir, f"libmcpx_{a.name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    shutil.rmtree(tmp, ignore_errors=True)
    print(lib)


if __name__ == "__main__":
    main()
