"""Build libdistraytracer.so (HIP, gfx950) in-tree with hipcc.

The shared library is the product: HIP kernels + host scene builder + C ABI
(include/distraytracer.h). It is built in-tree so it travels to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB_DIR = PKG / "lib"
LIB_PATH = LIB_DIR / "libdistraytracer.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["trace.hip", "render_minreg.hip", "photon_build.hip", "cli_loader.cpp", "scene_build.cpp", "photon.cpp"]
# per-source compiler flags: render_minreg.hip holds C3's and C5's render variants, which run
# faster with the register-minimising scheduler (C4's variant, in trace.hip, runs slower with it)
SOURCE_FLAGS = {"render_minreg.hip": ["-Xarch_device", "-mllvm=--amdgpu-sched-strategy=iterative-minreg",
                                      "-Xarch_device", "-mllvm=--amdgpu-use-amdgpu-trackers=1"]}
HEADERS = ["rt_types.h", "rt_internal.h", "host_math.h", "trace_device.h", "trace_kernels.h", "qdiv.h", "jfdlibm.h"]
# -ffp-contract=off: keep the reference's (Java) unfused double arithmetic so discrete
# decisions (hits, shadows, TIR) match the oracle; no fast-math (IEEE Inf/NaN needed).
COMPILE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
                 "-Wall", "-Wno-unused-result", "-Wno-unused-function"]


def _stale() -> bool:
    if not LIB_PATH.exists():
        return True
    t = LIB_PATH.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + HEADERS] + [PKG.parent / "include" / "distraytracer.h"]
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = False, defines: list[str] | None = None, out: Path | None = None) -> Path:
    """Build the library (in-tree). `defines`/`out`: tuning experiments (tools/variant_sweep.py)."""
    target = Path(out) if out else LIB_PATH
    if not force and not defines and out is None and not _stale():
        return LIB_PATH
    target.parent.mkdir(parents=True, exist_ok=True)
    tmp = target.with_suffix(".so.tmp%d" % os.getpid())
    objs, logs = [], []
    tag = "" if out is None else target.stem + "."
    for src in SOURCES:  # .hip -> device+host; .cpp -> host-only C++ (no device pass)
        obj = target.parent / (tag + src + ".o")
        lang = [] if src.endswith(".hip") else ["-x", "c++"]
        # defines starting with "-" are extra compiler flags, "@<source>:<flag>" a flag for one
        # source only (tuning experiments)
        dflags = []
        for d in defines or []:
            if d.startswith("@"):
                s, f = d[1:].split(":", 1)
                dflags += [f] if s == src else []
            else:
                dflags.append(d if d.startswith("-") else "-D" + d)
        cmd = [HIPCC, *COMPILE_FLAGS, *SOURCE_FLAGS.get(src, []), *dflags, *lang, "-c", str(CSRC / src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        logs.append(r.stderr)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n" + r.stderr[-4000:])
        objs.append(str(obj))
    r = subprocess.run([HIPCC, "-shared", "--offload-arch=gfx950", "-o", str(tmp), *objs], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stderr[-4000:])
    if verbose:
        print("\n".join(logs))
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    print(build(force=True))
