"""Build libdistraytracer.so (HIP, gfx950) in-tree with hipcc.

The shared library is the product: HIP kernels + host scene builder + C ABI
(include/distraytracer.h). It is built in-tree so it travels to the GPU box.

Provenance: the build id is a hash of every source and header compiled into the library, the
public header, and the compiler flags (this file's settings). It is compiled in (rt_build_id())
and written next to the library (lib/libdistraytracer.buildinfo.json); a library whose id
differs from the tree's is rebuilt, so a shipped .so is used only when it was built from these
sources with these flags. build() reports whether it compiled or reused the library.

Objects are cached by content (lib/obj/<source>.<hash>.o, the hash over the source, every header and
the flags): a rebuild compiles only the translation units whose inputs changed. The build id itself is
compiled into build_id.cpp alone.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB_DIR = PKG / "lib"
LIB_PATH = LIB_DIR / "libdistraytracer.so"
INFO_PATH = LIB_DIR / "libdistraytracer.buildinfo.json"
PUBLIC_HEADER = PKG.parent / "include" / "distraytracer.h"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["trace.hip", "render_minreg.hip", "photon_build.hip", "group.hip", "comm.hip", "cli_loader.cpp", "scene_build.cpp",
           "photon.cpp", "build_id.cpp"]
OBJ_DIR = LIB_DIR / "obj"
# per-source compiler flags: render_minreg.hip holds C3's and C5's render variants, which run
# faster with the register-minimising scheduler (C4's variant, in trace.hip, runs slower with it)
SOURCE_FLAGS = {"render_minreg.hip": ["-Xarch_device", "-mllvm=--amdgpu-sched-strategy=iterative-minreg",
                                      "-Xarch_device", "-mllvm=--amdgpu-use-amdgpu-trackers=1"]}
HEADERS = ["rt_types.h", "rt_internal.h", "comm.h", "host_math.h", "trace_device.h", "trace_kernels.h", "wavefront.h", "qdiv.h",
           "jfdlibm.h"]
# -ffp-contract=off: keep the reference's (Java) unfused double arithmetic so discrete
# decisions (hits, shadows, TIR) match the oracle; no fast-math (IEEE Inf/NaN needed).
COMPILE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
                 "-Wall", "-Wno-unused-result", "-Wno-unused-function"]

last_action = None  # "compiled" / "reused" after build()


def _extra_flags(src: str, defines: list[str] | None) -> list[str]:
    """Tuning-build flags for one source: "-..." is a compiler flag, "@<source>:<flag>" a flag
    for that source only, anything else a -D define. A per-source -D could give the two render
    translation units different struct layouts or LDS sizes, so it is refused."""
    out = []
    for d in defines or []:
        if d.startswith("@"):
            s, f = d[1:].split(":", 1)
            if f.startswith("-D"):
                raise ValueError(f"per-source defines are not allowed ({d}): both render TUs must agree")
            out += [f] if s == src else []
        else:
            out.append(d if d.startswith("-") else "-D" + d)
    return out


def build_id(defines: list[str] | None = None) -> str:
    """Hash of the sources, headers and flags a build compiles (16 hex digits)."""
    h = hashlib.sha256()
    for p in [CSRC / s for s in SOURCES + HEADERS] + [PUBLIC_HEADER]:
        h.update(p.name.encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(json.dumps([COMPILE_FLAGS, SOURCE_FLAGS, sorted(defines or [])]).encode())
    return h.hexdigest()[:16]


def built_id() -> str | None:
    """The build id recorded for the in-tree library, None if there is none."""
    try:
        return json.loads(INFO_PATH.read_text()).get("build_id") if LIB_PATH.exists() else None
    except (OSError, ValueError):
        return None


def _stale() -> bool:
    return built_id() != build_id()


def build(force: bool = False, verbose: bool = False, defines: list[str] | None = None, out: Path | None = None) -> Path:
    """Build the library (in-tree). `defines`/`out`: tuning experiments (tools/variant_sweep.py)."""
    global last_action
    target = Path(out) if out else LIB_PATH
    if not force and not defines and out is None and not _stale():
        last_action = "reused"
        return LIB_PATH
    bid = build_id(defines)
    target.parent.mkdir(parents=True, exist_ok=True)
    tmp = target.with_suffix(".so.tmp%d" % os.getpid())
    objs, procs = [], []
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hdr = b"".join(p.name.encode() + b"\0" + p.read_bytes() for p in [CSRC / h for h in HEADERS] + [PUBLIC_HEADER])
    for src in SOURCES:  # .hip -> device+host; .cpp -> host-only C++ (no device pass); compiled in parallel
        lang = [] if src.endswith(".hip") else ["-x", "c++"]
        flags = [*COMPILE_FLAGS, *SOURCE_FLAGS.get(src, []), *_extra_flags(src, defines)]
        if src == "build_id.cpp":
            flags.append(f'-DRT_BUILD_ID="{bid}"')
        key = hashlib.sha256((CSRC / src).read_bytes() + hdr + json.dumps([HIPCC, flags, lang]).encode()).hexdigest()[:16]
        obj = OBJ_DIR / f"{src}.{key}.o"
        objs.append(str(obj))
        if obj.exists() and not force:
            continue
        tmpo = obj.with_suffix(".o.tmp%d" % os.getpid())
        cmd = [HIPCC, *flags, *lang, "-c", str(CSRC / src), "-o", str(tmpo)]
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True), tmpo, obj))
    logs, failed = [], None
    for src, pr, tmpo, obj in procs:
        err = pr.communicate()[1]
        logs.append(err)
        if pr.returncode != 0:
            if failed is None:
                failed = f"hipcc failed on {src}:\n" + err[-4000:]
        else:
            os.replace(tmpo, obj)
    if failed:
        raise RuntimeError(failed)
    r = subprocess.run([HIPCC, "-shared", "--offload-arch=gfx950", "-o", str(tmp), *objs, "-ldl"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stderr[-4000:])
    if verbose:
        print("\n".join(logs))
    os.replace(tmp, target)
    for src in SOURCES:  # keep the newest few cached objects per source
        old = sorted(OBJ_DIR.glob(f"{src}.*.o"), key=lambda q: q.stat().st_mtime, reverse=True)
        for q in old[6:]:
            q.unlink(missing_ok=True)
    if out is None:
        INFO_PATH.write_text(json.dumps({"build_id": bid, "defines": defines or []}) + "\n")
    last_action = "compiled"
    return target


if __name__ == "__main__":
    print(build(force=True), last_action, build_id())
