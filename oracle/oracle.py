"""ORACLE / TEST INFRASTRUCTURE ONLY.

ctypes binding of the CPU restatement (oracle/src/oracle.cpp) of the
reference's per-pixel trace loop. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker.

Parity status (see DESIGN.md "Oracle"): the Java reference cannot be built or
run in this container (no JDK), so the restatement is pinned by the
hand-derived known-answer pixels of SURVEY.md 8(c) and by golden fixtures it
generates (tests/golden/, script tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "build" / "liboracle.so"

ST_NAMES = ["camera", "shadow", "refl", "refr", "box", "tri", "quad", "sphere", "light", "photon", "texel"]

_lib = None


def build(force: bool = False) -> Path:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off). make rebuilds only when a
    source is newer than the library; on the GPU box (no compiler run wanted) a present library
    is used as shipped."""
    src_newer = LIB_PATH.exists() and any(
        f.stat().st_mtime > LIB_PATH.stat().st_mtime
        for f in [*(ORACLE_DIR / "src").iterdir(), ORACLE_DIR.parent / "distraytracer_old_amd" / "csrc" / "jfdlibm.h"])
    if force or not LIB_PATH.exists() or src_newer:
        subprocess.run(["make", "-C", str(ORACLE_DIR)] + (["-B"] if force else []), check=True, capture_output=True)
    return LIB_PATH


def lib():
    """ORACLE_LIB overrides the library (the sanitizer build, tools/sanitize.sh)."""
    global _lib
    if _lib is None:
        path = os.environ.get("ORACLE_LIB")
        if not path:
            build()
        L = ctypes.CDLL(path or str(LIB_PATH))
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_register_texture.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_load.restype = ctypes.c_void_p
        L.oracle_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_build_photons.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_photons.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int]
        L.oracle_set_photons.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.oracle_math_eval.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.oracle_camera_hits.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.oracle_knn.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def math_eval(x) -> np.ndarray:
    """Host fdlibm sin / cos / asin / acos (the oracle's, csrc/jfdlibm.h): [n, 4] float64."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros((len(x), 4), dtype=np.float64)
    lib().oracle_math_eval(x.ctypes.data, out.ctypes.data, len(x))
    return out


class OracleScene:
    """A .cli scene loaded by the oracle's own loader (myRTFileReader restatement)."""

    def __init__(self, scene_dir: str | os.PathLike, cli: str, textures: dict | None = None):
        L = lib()
        for name, arr in (textures or {}).items():
            a = np.ascontiguousarray(arr, dtype=np.uint8)
            L.oracle_register_texture(name.encode(), a.shape[1], a.shape[0], a.ctypes.data)
        self._h = L.oracle_load(str(scene_dir).encode(), cli.encode())
        if not self._h:
            raise RuntimeError("oracle load failed: " + L.oracle_last_error().decode())

    def info(self) -> dict:
        v = np.zeros(8, dtype=np.int64)
        lib().oracle_info(self._h, v.ctypes.data, 8)
        keys = ["objects", "lights", "bvh_internal", "bvh_leaves", "bvh_depth", "bvh_prims", "prims", "rays_per_pixel"]
        return dict(zip(keys, v.tolist()))

    def build_photons(self, seed: int) -> int:
        return lib().oracle_build_photons(self._h, seed)

    def set_photons(self, pos, pwr):
        """Install a photon_list (insertion order) and build the oracle's kd-tree over it."""
        pos = np.ascontiguousarray(pos, dtype=np.float64)
        pwr = np.ascontiguousarray(pwr, dtype=np.float64)
        lib().oracle_set_photons(self._h, pos.ctypes.data, pwr.ctypes.data, len(pos))

    def photons(self):
        """(pos [n,3], pwr [n,3]) of the photon map in insertion order (after build_photons)."""
        n = lib().oracle_photons(self._h, None, None, 0)
        pos = np.zeros((n, 3)); pwr = np.zeros((n, 3))
        lib().oracle_photons(self._h, pos.ctypes.data, pwr.ctypes.data, n)
        return pos, pwr

    def render(self, W: int, H: int, spp: int = 0, seed: int = 0x5EED0001, rows=None, row_step: int = 1,
               threads: int = 0):
        """Returns (rgb float32 [n,W,3], argb int32 [n,W], stats dict) for rows[0]:rows[1]:row_step."""
        r0, r1 = (0, H) if rows is None else rows
        n = len(range(r0, r1, row_step))
        rgb = np.zeros((n, W, 3), dtype=np.float32)
        argb = np.zeros((n, W), dtype=np.int32)
        st = np.zeros(16, dtype=np.uint64)
        nt = threads if threads > 0 else min(16, os.cpu_count() or 1)  # GPU box CPU share is 16
        rc = lib().oracle_render(self._h, W, H, spp, seed, r0, r1, row_step, rgb.ctypes.data, argb.ctypes.data,
                                 st.ctypes.data, nt)
        if rc != 0:
            raise RuntimeError("oracle render failed")
        return rgb, argb, dict(zip(ST_NAMES, st[: len(ST_NAMES)].tolist()))

    def knn(self, p, cap: int = 4096):
        """find_near's neighbourhood of point p: (photon indices in poll order, farthest first; d2)."""
        idx = np.zeros(cap, dtype=np.int32)
        d2 = np.zeros(cap, dtype=np.float64)
        n = lib().oracle_knn(self._h, float(p[0]), float(p[1]), float(p[2]), idx.ctypes.data, d2.ctypes.data, cap)
        return idx[:min(n, cap)].copy(), d2[:min(n, cap)].copy()

    def camera_hits(self, W: int, H: int, threads: int = 0) -> np.ndarray:
        """uint8 [H, W]: 1 where the un-jittered FOV camera ray hits an object, 0 where it
        falls through to the background / skydome (myScene.java:907-914)."""
        m = np.zeros((H, W), dtype=np.uint8)
        nt = threads if threads > 0 else min(16, os.cpu_count() or 1)
        if lib().oracle_camera_hits(self._h, W, H, m.ctypes.data, nt) != 0:
            raise RuntimeError("oracle_camera_hits: " + lib().oracle_last_error().decode())
        return m

    def close(self):
        if self._h:
            lib().oracle_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
