"""In-tree build of the HIP extension libmcpx.so (gfx950 only).

    python -m mcp_amd.build            # build if sources are newer than the .so
    python -m mcp_amd.build --force

Both translation units are compiled with -ffp-contract=off: the kernels'
arithmetic contract (explicit fma only) is what makes them bit-identical to
the oracle.  hipcc cross-compiles for gfx950 without a GPU present.
"""

from __future__ import annotations

import glob
import hashlib
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmcpx.so")
SOURCES = [os.path.join(CSRC, f) for f in (
    "ipm_inst_red_qp.hip", "ipm_inst_spec.hip", "ipm_inst_schur_qp.hip", "ipm_inst_schur_aff.hip", "ipm_inst_red_aff.hip",
    "ipm_inst_dense_qp.hip", "ipm_inst_dense_aff.hip", "sens_inst_vjp.hip", "sens_inst_jvp.hip",
    "ipm_inst_wg.hip", "ipm_inst_wg_vr.hip", "ipm_inst_wg_gj.hip", "sens_inst_wg.hip", "ipm_inst_fused.hip", "mcpx_api.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("ipm_kernel.h", "ipm_kernel_impl.hpp", "bcast_group.inc", "sens_kernel.h", "sens_kernel_impl.hpp",
    "ipm_wg.h", "ipm_wg_impl.hpp", "lu_vr.hpp", "gj_vr.hpp", "sens_wg_impl.hpp")] + [
    os.path.join(ROOT, "include", "mcpx.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -amdgpu-mfma-vgpr-form: MFMA accumulators in arch VGPRs (dead during the LU)
# instead of AGPRs, which would add to every wave's register allocation.
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC",
         "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


STAMP = LIB + ".srchash"


def source_hash(extra_flags=()) -> str:
    """sha256 over the text of every source the library is built from and the
    compiler flags: the identity of a build (written next to the .so, quoted by
    the profile summaries so that bench.py only cites evidence of this build)."""
    h = hashlib.sha256()
    for p in DEPS:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0" + open(p, "rb").read() + b"\0")
    h.update(" ".join([HIPCC.rsplit("/", 1)[-1], *FLAGS, *extra_flags]).encode())
    return h.hexdigest()[:16]


def built_hash() -> str | None:
    """source_hash() recorded when mcp_amd/libmcpx.so was built, or None."""
    try:
        return open(STAMP).read().strip() or None
    except OSError:
        return None


def _stale() -> bool:
    # content, not mtimes: a snapshot copied to another machine keeps its stamp only
    # if it was built from exactly these sources with these flags
    return not os.path.exists(LIB) or built_hash() != source_hash()


# Per-translation-unit object cache of this container (never shipped): a TU is recompiled
# only when its text, a file it includes (transitively) or the flags change.
OBJ_CACHE = os.environ.get("MCPX_OBJ_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "mcpx_objs")
_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _tu_key(src: str, flags) -> str:
    h = hashlib.sha256(" ".join([HIPCC, *flags]).encode())
    seen, todo = set(), [os.path.abspath(src)]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.add(f)
        text = open(f, "rb").read()
        h.update(os.path.relpath(f, ROOT).encode() + b"\0" + text + b"\0")
        todo += [os.path.normpath(os.path.join(os.path.dirname(f), inc))
                 for inc in _INCLUDE.findall(text.decode(errors="replace"))]
    return h.hexdigest()[:24]


def build(force: bool = False, verbose: bool = False, extra_flags=(), out: str | None = None) -> str:
    """`out`: alternative output path (kernel A/B variants built with `extra_flags`)."""
    lib_path = out or LIB
    if out is None and not force and not _stale():
        return LIB
    t0 = time.time()
    stamp = source_hash(extra_flags)  # of the sources as they are when the compiles start
    objs, procs = [], []
    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(SOURCES), os.cpu_count() or 1)
    tmp_dir = tempfile.mkdtemp(prefix="mcpx_build_")
    built = []  # (cache dir, tmp object) of the TUs compiled in this call
    for src in SOURCES:  # one hipcc per translation unit, `jobs` at a time
        base = os.path.basename(src)
        obj = os.path.join(tmp_dir, base + ".o")
        cdir = os.path.join(OBJ_CACHE, base + "." + _tu_key(src, [*FLAGS, *extra_flags]))
        objs.append(obj)
        if not force and os.path.exists(os.path.join(cdir, "ok")):  # object + device .s of an identical TU
            for f in os.listdir(cdir):
                if f != "ok":
                    shutil.copy2(os.path.join(cdir, f), os.path.join(tmp_dir, f))
            if verbose:
                print(f"cached {base}", flush=True)
            continue
        # -save-temps=obj keeps the device .s next to the object for the hazard check
        cmd = [HIPCC, *FLAGS, *extra_flags, "-save-temps=obj", "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), src))
        built.append((cdir, src))
        while sum(p.poll() is None for p, _ in procs) >= jobs:
            time.sleep(0.2)
    for p, src in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, f"hipcc {src}")
    for cdir, src in built:
        base = os.path.basename(src)
        stem = os.path.splitext(base)[0]
        try:
            os.makedirs(cdir, exist_ok=True)
            for f in os.listdir(tmp_dir):
                if f == base + ".o" or (f.startswith(stem + "-hip-amdgcn") and f.endswith(".s")):
                    shutil.copy2(os.path.join(tmp_dir, f), os.path.join(cdir, f))
            open(os.path.join(cdir, "ok"), "w").close()
        except OSError:
            pass  # the cache is an accelerator only
    # hipcc does not pad hazards whose reader sits inside inline asm: refuse a build in
    # which a compiler-placed VALU write feeds a DPP / cross-lane asm read too early
    checker = os.path.join(ROOT, "tools", "check_dpp_hazards.py")
    asms = sorted(glob.glob(os.path.join(tmp_dir, "*amdgcn*gfx950.s")))
    if not os.path.exists(checker):
        raise RuntimeError(f"the inline-asm hazard checker {checker} is missing: refusing an unchecked build")
    if len(asms) < sum(1 for s in SOURCES if s.endswith(".hip")):  # every kernel TU leaves its device .s
        raise RuntimeError(f"found {len(asms)} device .s files under {tmp_dir} for the hazard check "
                           "(-save-temps naming changed?): refusing an unchecked build")
    for asm in asms:
        r = subprocess.run([sys.executable, checker, asm], capture_output=True, text=True)
        if verbose:
            print(f"{os.path.basename(asm)}: {r.stdout.strip().splitlines()[-1]}", flush=True)
        if r.returncode != 0:
            raise RuntimeError(f"inline-asm hazard in {asm}:\n{r.stdout[-2000:]}")
    tmp = lib_path + ".tmp"
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], check=True)
    os.replace(tmp, lib_path)
    if out is None:
        with open(STAMP, "w") as f:
            f.write(stamp + "\n")
    shutil.rmtree(tmp_dir, ignore_errors=True)
    if verbose:
        print(f"built {lib_path} in {time.time() - t0:.1f}s", flush=True)
    return lib_path


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True,
          extra_flags=["-Rpass-analysis=kernel-resource-usage"] if "--resources" in sys.argv else [])
