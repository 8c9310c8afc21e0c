"""ctypes binding of libdistraytracer.so (include/distraytracer.h).

This is the product path: every render goes through the HIP kernels. There is
no CPU fallback -- if the library is missing or no GPU is visible the calls
raise RTError.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

from . import build as _build
from .scenes import SCENE_DIR, prepare

ST_NAMES = ["camera", "shadow", "refl", "refr", "box", "tri", "quad", "implicit", "light", "photon", "texel",
            "node", "leaf", "member", "root", "top",
            # the same record loads counted per wave step where a wave loads a record once for all
            # its lanes (RT_ST_W_*, include/distraytracer.h)
            "w_node", "w_tri", "w_quad", "w_implicit", "w_light", "w_photon"]
RT_ST_N = 24
INFO_NAMES = ["objects", "lights", "bvh_internal", "bvh_leaves", "bvh_depth", "bvh_prims", "prims",
              "rays_per_pixel", "device_bytes", "triangles", "photons", "materials", "photon_mode",
              "photon_count"]


class RTError(RuntimeError):
    pass


class TextureDesc(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int32), ("h", ctypes.c_int32), ("rgb", ctypes.c_void_p)]


class RenderParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("row0", ctypes.c_int32), ("row1", ctypes.c_int32), ("row_step", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("flags", ctypes.c_uint32), ("row_band", ctypes.c_int32)]


EXPORTS = ["rt_abi_version", "rt_build_id", "rt_last_error", "rt_device_count", "rt_scene_create", "rt_scene_load_cli",
           "rt_scene_inspect_cli",
           "rt_scene_info", "rt_scene_destroy", "rt_photons_build", "rt_render", "rt_render_device",
           "rt_render_count", "rt_time_render", "rt_render_pass", "rt_refine_steps", "rt_scene_photons",
           "rt_scene_photon_map", "rt_photons_shoot",
           "rt_photons_set",
           "rt_png_name", "rt_scene_save_name", "rt_math_eval", "rt_tile_layout", "rt_tile_costs",
           "rt_render_tiles_device", "rt_render_tiles_count",
           "rt_render_pixels_device", "rt_photon_gather",
           "rt_photon_kdtree", "rt_scene_photon_kdtree",
           # ABI 6: the multi-GPU frame (rt_group_*), the kernel variants
           "rt_render_variant", "rt_rank_plan", "rt_group_unique_id", "rt_group_create", "rt_group_create_rank", "rt_group_render",
           "rt_group_sync", "rt_group_render_host", "rt_group_frame", "rt_group_info", "rt_group_plan",
           "rt_group_rank_pixels", "rt_group_kernel_ms", "rt_group_time_rank", "rt_group_count", "rt_group_rebalance",
           "rt_group_destroy", "rt_group_rccl_selftest",
           # ABI 7: communicators (RCCL / caller host transport), the group and the photon pre-pass over them
           "rt_comm_create_rccl", "rt_comm_create_host", "rt_comm_info", "rt_comm_destroy", "rt_comm_selftest",
           "rt_group_create_comm",
           "rt_photons_build_comm", "rt_photons_build_local"]

_lib = None


def lib_path() -> Path:
    """The in-tree library; DISTRAYTRACER_LIB overrides it (tuning builds, tools/variant_sweep.py)."""
    env = os.environ.get("DISTRAYTRACER_LIB")
    return Path(env) if env else _build.LIB_PATH


def lib():
    """Load the HIP library; raises RTError (never falls back) if it is absent."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch ships its own libamdhip64 (soname libamdhip64.so.7,
        # loaded by file name), and a process that loads ours (/opt/rocm's, same soname) first and
        # torch's later holds two runtimes, the second of which sees no GPU. With torch imported
        # first the library binds to the runtime already loaded (the soname matches).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        p = lib_path()
        if not p.exists():
            raise RTError(f"{p} is missing: build it with `python -m distraytracer_old_amd.build`")
        L = ctypes.CDLL(str(p))
        L.rt_last_error.restype = ctypes.c_char_p
        if hasattr(L, "rt_build_id"):  # ABI >= 5 (older tuning builds lack it: build_id() -> "unknown")
            L.rt_build_id.restype = ctypes.c_char_p
        L.rt_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.rt_scene_load_cli.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(TextureDesc),
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.rt_scene_inspect_cli.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(TextureDesc),
                                           ctypes.c_void_p, ctypes.c_int]
        L.rt_scene_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.rt_scene_destroy.argtypes = [ctypes.c_void_p]
        L.rt_photons_build.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.rt_scene_photons.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.POINTER(ctypes.c_int64)]
        L.rt_scene_photon_map.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.c_int32)]
        L.rt_photons_shoot.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.rt_refine_steps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.rt_render_pass.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.rt_photons_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.rt_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_void_p]
        L.rt_render_count.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.rt_render_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.rt_time_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double)]
        L.rt_tile_layout.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p]
        L.rt_tile_costs.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_int]
        L.rt_render_tiles_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.rt_render_pixels_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.rt_render_tiles_count.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams), ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p]
        L.rt_photon_kdtree.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.rt_scene_photon_kdtree.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.rt_photon_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.rt_math_eval.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        L.rt_png_name.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.rt_scene_save_name.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        if hasattr(L, "rt_group_create"):  # ABI >= 6
            vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
            L.rt_rank_plan.argtypes = [vp, vp, i32, i32, dbl, i32, vp, vp]
            L.rt_group_rebalance.argtypes = [vp, i32, i32, vp]
            L.rt_render_variant.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_uint32)]
            L.rt_group_unique_id.argtypes = [vp, i32]
            L.rt_group_create.argtypes = [vp, i32, ctypes.POINTER(RenderParams), ctypes.c_uint32, dbl, i32,
                                          ctypes.POINTER(vp)]
            L.rt_group_create_rank.argtypes = [vp, i32, i32, vp, ctypes.POINTER(RenderParams), ctypes.c_uint32, dbl,
                                               i32, ctypes.POINTER(vp)]
            L.rt_group_render.argtypes = [vp, vp, vp]
            L.rt_group_sync.argtypes = [vp]
            L.rt_group_render_host.argtypes = [vp, vp, vp]
            L.rt_group_frame.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
            L.rt_group_info.argtypes = [vp, vp, i32]
            L.rt_group_plan.argtypes = [vp, vp, vp, i32]
            L.rt_group_rank_pixels.argtypes = [vp, i32, vp, i64]
            L.rt_group_kernel_ms.argtypes = [vp, i32, ctypes.POINTER(dbl), ctypes.POINTER(i32)]
            L.rt_group_time_rank.argtypes = [vp, i32, i32, i32, ctypes.POINTER(dbl), ctypes.POINTER(dbl)]
            L.rt_group_count.argtypes = [vp, i32, vp]
            L.rt_group_destroy.argtypes = [vp]
            L.rt_group_destroy.restype = None
            L.rt_group_rccl_selftest.argtypes = [i32, i32]
        if hasattr(L, "rt_comm_create_host"):  # ABI >= 7
            vp, i32, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
            L.rt_comm_create_rccl.argtypes = [i32, i32, vp, i32, ctypes.POINTER(vp)]
            L.rt_comm_create_host.argtypes = [i32, i32, ctypes.POINTER(CommOps), ctypes.POINTER(vp)]
            L.rt_comm_info.argtypes = [vp, vp, i32]
            L.rt_comm_destroy.argtypes = [vp]
            L.rt_comm_destroy.restype = None
            L.rt_comm_selftest.argtypes = [vp, i32]
            L.rt_group_create_comm.argtypes = [vp, vp, ctypes.POINTER(RenderParams), ctypes.c_uint32, dbl, i32,
                                               ctypes.POINTER(vp)]
            L.rt_photons_build_comm.argtypes = [vp, vp, ctypes.c_uint64]
            L.rt_photons_build_local.argtypes = [vp, i32, ctypes.c_uint64]
        _lib = L
    return _lib


def _name_call(fn, *args) -> str:
    n = fn(*args, None, 0)
    if n < 0:
        raise RTError(f"{fn.__name__} failed ({n}): {lib().rt_last_error().decode()}")
    buf = ctypes.create_string_buffer(n + 1)
    fn(*args, buf, n + 1)
    return buf.value.decode()


def build_id() -> str:
    """The loaded library's build id (rt_build_id: hash of its sources and flags, build.py)."""
    return lib().rt_build_id().decode() if hasattr(lib(), "rt_build_id") else "unknown"


def png_name(save_name: str) -> str:
    """myScene.saveFile's image name for a `write` argument (myScene.java:1185-1196)."""
    return _name_call(lib().rt_png_name, save_name.encode())


def _check(rc: int, what: str):
    if rc != 0:
        raise RTError(f"{what} failed ({rc}): {lib().rt_last_error().decode()}")


def math_eval(x, device: int = 0) -> np.ndarray:
    """Device fdlibm sin / cos / asin / acos of x (diagnostics, rt_math_eval): [n, 4] float64."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros((len(x), 4), dtype=np.float64)
    _check(lib().rt_math_eval(x.ctypes.data, out.ctypes.data, len(x), device), "rt_math_eval")
    return out


def photon_kdtree(pos) -> np.ndarray:
    """The reference's kd-tree over a photon_list (host-only, rt_photon_kdtree): int32 [n, 4] =
    (photon list index, axis, left, right) per node, DFS pre-order."""
    pos = np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
    out = np.zeros((len(pos), 4), dtype=np.int32)
    _check(lib().rt_photon_kdtree(pos.ctypes.data, len(pos), out.ctypes.data), "rt_photon_kdtree")
    return out


def rank_plan(cost, world: int, heavy: float = 0.0, slots: int = 0, weight=None):
    """The deterministic multi-GPU plan of a layout's tile costs (rt_rank_plan, host only):
    (owner int32 [ntiles], order int32 [ntiles]) -- owner[t] in [0, world) renders tile t in its wave
    run, world + r marks one of rank r's split (one sample per wave) tiles; order = dispatch order.
    weight: per-tile cut factors (the runs hold equal sums of cost x weight)."""
    c = np.ascontiguousarray(cost, dtype=np.uint32)
    w = None if weight is None else np.ascontiguousarray(weight, dtype=np.float64)
    if w is not None and w.shape != c.shape:  # the C side reads weight[t] for every tile
        raise ValueError(f"rank_plan: weight has {w.size} entries, cost {c.size}")
    owner = np.zeros(len(c), dtype=np.int32)
    order = np.zeros(len(c), dtype=np.int32)
    _check(lib().rt_rank_plan(c.ctypes.data, None if w is None else w.ctypes.data, len(c), world, heavy, slots,
                              owner.ctypes.data, order.ctypes.data), "rt_rank_plan")
    return owner, order


def group_unique_id() -> bytes:
    """128-byte RCCL unique id for rt_group_create_rank (call on rank 0, share with the others)."""
    buf = ctypes.create_string_buffer(128)
    n = lib().rt_group_unique_id(buf, 128)
    if n < 0:
        raise RTError(f"rt_group_unique_id failed ({n}): {lib().rt_last_error().decode()}")
    return buf.raw[:n]


def rccl_selftest(device: int = 0, n: int = 4099) -> None:
    """rt_group_rccl_selftest: every RCCL call of the group's transport through a one-rank
    communicator on `device` (bindings check for one-GPU machines); raises RTError on a failure."""
    _check(lib().rt_group_rccl_selftest(device, n), "rt_group_rccl_selftest")


GROUP_RGB = 1  # RT_GROUP_RGB: exchange the float-RGB plane too
GROUP_COPY = 2  # RT_GROUP_COPY: device copies in one process (ranks may share a device)
GROUP_INFO = ["world", "local_ranks", "first_rank", "ntiles", "tiles_x", "tw", "th", "rccl", "frames", "plan_checks"]
TRANSPORT_NAMES = {0: "copy", 1: "rccl", 2: "host"}

# rt_comm_ops (include/distraytracer.h): the host transport's four blocking callbacks
_BCAST = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int)
_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
_SEND = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int)
_RECV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int)


class CommOps(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("bcast", _BCAST), ("allgather", _ALLGATHER), ("send", _SEND),
                ("recv", _RECV)]


def _host_bytes(addr: int, n: int):
    """A writable uint8 torch view of n host bytes at addr (no copy)."""
    import torch

    return torch.frombuffer((ctypes.c_uint8 * n).from_address(addr), dtype=torch.uint8)


class Comm:
    """A communicator (rt_comm_*): RCCL (`rccl`) or the host transport (`host`) whose collectives
    are torch.distributed calls on CPU tensors (gloo) -- the caller's-own-transport path, which lets
    the ranks of one-process-per-GPU groups share a device."""

    def __init__(self, handle, keep=None):
        self._h = handle
        self._keep = keep  # the callbacks (ctypes must keep them alive while the library may call them)

    @classmethod
    def rccl(cls, rank: int, world: int, uid, device: int) -> "Comm":
        h = ctypes.c_void_p()
        u = ctypes.create_string_buffer(bytes(uid), 128) if uid is not None else None
        _check(lib().rt_comm_create_rccl(rank, world, u, device, ctypes.byref(h)), "rt_comm_create_rccl")
        return cls(h)

    @classmethod
    def host(cls, dist, group=None) -> "Comm":
        """Host transport over an initialised torch.distributed process group (gloo: CPU tensors)."""
        import torch

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        errors = []

        def guard(fn):
            def call(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # reported as RT_E_HIP by the library; the message kept here
                    errors.append(repr(e))
                    return 1
            return call

        def bcast(_ctx, buf, n, root):
            dist.broadcast(_host_bytes(buf, n), root, group=group)

        def allgather(_ctx, inp, out, n):
            src = _host_bytes(inp, n).clone()
            outs = [torch.empty(n, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(outs, src, group=group)
            _host_bytes(out, n * world).copy_(torch.cat(outs))

        def send(_ctx, buf, n, peer):
            dist.send(_host_bytes(buf, n).clone(), peer, group=group)

        def recv(_ctx, buf, n, peer):
            t = torch.empty(n, dtype=torch.uint8)
            dist.recv(t, peer, group=group)
            _host_bytes(buf, n).copy_(t)

        cbs = (_BCAST(guard(bcast)), _ALLGATHER(guard(allgather)), _SEND(guard(send)), _RECV(guard(recv)))
        ops = CommOps(None, *cbs)
        h = ctypes.c_void_p()
        _check(lib().rt_comm_create_host(rank, world, ctypes.byref(ops), ctypes.byref(h)), "rt_comm_create_host")
        c = cls(h, (cbs, ops))
        c.errors = errors
        return c

    def selftest(self, n: int = 1031):
        """rt_comm_selftest: all-gather, a broadcast from every rank and (host transport) the group's
        send / receive pattern, checked on the host (collective). Raises RTError on a failure."""
        rc = lib().rt_comm_selftest(self._h, n)
        if rc != 0:
            extra = f" (callback errors: {self.errors})" if getattr(self, "errors", None) else ""
            raise RTError(f"rt_comm_selftest failed ({rc}): {lib().rt_last_error().decode()}{extra}")

    def info(self) -> dict:
        v = np.zeros(4, dtype=np.int64)
        _check(lib().rt_comm_info(self._h, v.ctypes.data, 4), "rt_comm_info")
        return {"rank": int(v[0]), "world": int(v[1]), "transport": TRANSPORT_NAMES.get(int(v[2]), "?"),
                "device": int(v[3])}

    def close(self):
        if self._h:
            lib().rt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def build_photons_local(scenes, seed: int):
    """rt_photons_build_local: the sharded photon pre-pass emulated in one process (scene q shoots
    shard q of len(scenes); scenes may repeat); every distinct scene gets the merged map."""
    arr = (ctypes.c_void_p * len(scenes))(*[s._h for s in scenes])
    _check(lib().rt_photons_build_local(arr, len(scenes), seed), "rt_photons_build_local")


class Group:
    """A multi-GPU frame (rt_group_*): one process driving N ranks (`create`) or one rank per
    process (`create_rank`). render() enqueues a frame; rank 0's frame lands in its own device
    buffers (frame()) or in caller-owned ones."""

    def __init__(self, handle, scenes):
        self._h = handle
        self._scenes = scenes  # keep the scenes alive while the group uses them

    @classmethod
    def create(cls, scenes, W, H, spp=0, seed=0x5EED0001, flags=0, rgb=False, copy=False, heavy=0.0, slots=0):
        p = params(W, H, spp, seed, None, 1, flags, 1)
        arr = (ctypes.c_void_p * len(scenes))(*[s._h for s in scenes])
        h = ctypes.c_void_p()
        gf = (GROUP_RGB if rgb else 0) | (GROUP_COPY if copy else 0)
        _check(lib().rt_group_create(arr, len(scenes), ctypes.byref(p), gf, heavy, slots, ctypes.byref(h)),
               "rt_group_create")
        return cls(h, list(scenes))

    @classmethod
    def create_comm(cls, scene, comm, W, H, spp=0, seed=0x5EED0001, flags=0, rgb=False, heavy=0.0, slots=0):
        """One rank of a one-process-per-GPU group over a communicator (rt_group_create_comm; collective).
        comm None: a one-rank group."""
        p = params(W, H, spp, seed, None, 1, flags, 1)
        h = ctypes.c_void_p()
        _check(lib().rt_group_create_comm(scene._h, comm._h if comm is not None else None, ctypes.byref(p),
                                          GROUP_RGB if rgb else 0, heavy, slots, ctypes.byref(h)),
               "rt_group_create_comm")
        return cls(h, [scene, comm])

    @classmethod
    def create_rank(cls, scene, rank, world, uid, W, H, spp=0, seed=0x5EED0001, flags=0, rgb=False, heavy=0.0,
                    slots=0):
        p = params(W, H, spp, seed, None, 1, flags, 1)
        h = ctypes.c_void_p()
        u = ctypes.create_string_buffer(bytes(uid), 128) if uid is not None else None
        _check(lib().rt_group_create_rank(scene._h, rank, world, u, ctypes.byref(p), GROUP_RGB if rgb else 0, heavy,
                                          slots, ctypes.byref(h)), "rt_group_create_rank")
        return cls(h, [scene])

    def render(self, rgb_ptr: int = 0, argb_ptr: int = 0):
        _check(lib().rt_group_render(self._h, ctypes.c_void_p(rgb_ptr or None), ctypes.c_void_p(argb_ptr or None)),
               "rt_group_render")

    def sync(self):
        _check(lib().rt_group_sync(self._h), "rt_group_sync")

    def render_host(self, W, H, rgb=True):
        """Blocking frame into host arrays (rank 0's process): (rgb [H, W, 3] float32 or None, argb [H, W])."""
        a = np.zeros((H, W), dtype=np.int32)
        c = np.zeros((H, W, 3), dtype=np.float32) if rgb else None
        _check(lib().rt_group_render_host(self._h, c.ctypes.data if rgb else None, a.ctypes.data),
               "rt_group_render_host")
        return c, a

    def frame(self):
        """Device pointers (rgb or 0, argb) of the group's own frame on rank 0's device."""
        r, a = ctypes.c_void_p(), ctypes.c_void_p()
        _check(lib().rt_group_frame(self._h, ctypes.byref(r), ctypes.byref(a)), "rt_group_frame")
        return r.value or 0, a.value or 0

    def info(self) -> dict:
        v = np.zeros(len(GROUP_INFO), dtype=np.int64)
        _check(lib().rt_group_info(self._h, v.ctypes.data, len(v)), "rt_group_info")
        return dict(zip(GROUP_INFO, v.tolist()))

    def plan(self):
        n = self.info()["ntiles"]
        owner = np.zeros(n, dtype=np.int32)
        order = np.zeros(n, dtype=np.int32)
        r = lib().rt_group_plan(self._h, owner.ctypes.data, order.ctypes.data, n)
        if r < 0:
            raise RTError(f"rt_group_plan: {lib().rt_last_error().decode()}")
        return owner, order

    def rank_tiles(self, rank: int):
        """(run tiles, split tiles) of a rank in dispatch order."""
        owner, order = self.plan()
        world = self.info()["world"]
        o = owner[order]
        return order[o == rank], order[o == world + rank]

    def rank_pixels(self, rank: int) -> np.ndarray:
        n = lib().rt_group_rank_pixels(self._h, rank, None, 0)
        if n < 0:
            raise RTError(f"rt_group_rank_pixels: {lib().rt_last_error().decode()}")
        out = np.zeros(n, dtype=np.int32)
        lib().rt_group_rank_pixels(self._h, rank, out.ctypes.data, n)
        return out

    def kernel_ms(self, rank: int):
        ms, fr = ctypes.c_double(0), ctypes.c_int(0)
        _check(lib().rt_group_kernel_ms(self._h, rank, ctypes.byref(ms), ctypes.byref(fr)), "rt_group_kernel_ms")
        return ms.value, fr.value

    def time_rank(self, rank: int, warmup: int = 3, iters: int = 20):
        """(wall ms per step, mean render ms) of one rank's pipelined step alone (RT_GROUP_COPY groups)."""
        a, b = ctypes.c_double(0), ctypes.c_double(0)
        _check(lib().rt_group_time_rank(self._h, rank, warmup, iters, ctypes.byref(a), ctypes.byref(b)),
               "rt_group_time_rank")
        return a.value, b.value

    def rebalance(self, rounds: int = 2, iters: int = 5):
        """Re-cut the plan from measured rank render times (rt_group_rebalance; collective in rank
        mode); returns the ranks' render ms after the last cut."""
        out = np.zeros(self.info()["world"], dtype=np.float64)
        _check(lib().rt_group_rebalance(self._h, rounds, iters, out.ctypes.data), "rt_group_rebalance")
        return out

    def count(self, rank: int) -> dict:
        st = np.zeros(RT_ST_N, dtype=np.uint64)
        _check(lib().rt_group_count(self._h, rank, st.ctypes.data), "rt_group_count")
        return dict(zip(ST_NAMES, st[: len(ST_NAMES)].tolist()))

    def close(self):
        if self._h:
            lib().rt_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(lib().rt_device_count(ctypes.byref(n)), "rt_device_count")
    return n.value


def _tex_args(textures: dict):
    names = list(textures)
    arrs = [np.ascontiguousarray(textures[n], dtype=np.uint8) for n in names]
    cnames = (ctypes.c_char_p * max(1, len(names)))(*[n.encode() for n in names])
    tds = (TextureDesc * max(1, len(names)))(*[TextureDesc(a.shape[1], a.shape[0], a.ctypes.data) for a in arrs])
    return names, arrs, cnames, tds


def inspect_cli(cli: str, scene_dir=SCENE_DIR, textures: dict | None = None) -> dict:
    """Host-only parse + flatten + BVH build (no GPU needed)."""
    if textures is None:
        textures = prepare(cli, Path(scene_dir))
    names, arrs, cnames, tds = _tex_args(textures)
    v = np.zeros(len(INFO_NAMES), dtype=np.int64)
    _check(lib().rt_scene_inspect_cli(str(scene_dir).encode(), cli.encode(), len(names), cnames, tds,
                                      v.ctypes.data, len(INFO_NAMES)), "rt_scene_inspect_cli")
    return dict(zip(INFO_NAMES, v.tolist()))


RENDER_GENERIC = 1  # RT_RENDER_GENERIC: the all-features kernel instead of the scene-specialised one
RENDER_ROWMAJOR = 2  # RT_RENDER_ROWMAJOR: row-major tile dispatch instead of the longest-first schedule
RENDER_NOCULL = 4  # RT_RENDER_NOCULL: no bounding-sphere culling of top-level primitives
RENDER_SHCOMPACT = 8  # RT_RENDER_SHCOMPACT: a wave's shadow rays traced compacted (same image)
RENDER_NOWAVECULL = 16  # RT_RENDER_NOWAVECULL: no wave-level shadow candidate test (same image)
RENDER_WAVEFRONT = 32  # RT_RENDER_WAVEFRONT: level-synchronous shading (same image)
RENDER_PIXEL_WAVES = 64  # RT_RENDER_PIXEL_WAVES: one pixel per wave (same image)


def params(W, H, spp=0, seed=0x5EED0001, rows=None, row_step=1, flags=0, row_band=1) -> RenderParams:
    r0, r1 = (0, H) if rows is None else rows
    return RenderParams(W, H, spp, r0, r1, row_step, seed, flags, row_band)


def nrows_of(p: RenderParams) -> int:
    """Rows row0 + k*row_step*row_band + j (0 <= j < row_band) below row1."""
    r1 = p.row1 if p.row1 > 0 else p.height
    step, band = max(1, p.row_step), max(1, p.row_band)
    full, rest = divmod(r1 - p.row0, step * band)
    return full * band + min(rest, band)


class Scene:
    """A scene resident on one GPU (rt_scene*)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load_cli(cls, cli: str, scene_dir=SCENE_DIR, textures: dict | None = None, device: int = 0) -> "Scene":
        if textures is None:
            textures = prepare(cli, Path(scene_dir))
        names, arrs, cnames, tds = _tex_args(textures)
        h = ctypes.c_void_p()
        _check(lib().rt_scene_load_cli(str(scene_dir).encode(), cli.encode(), len(names), cnames, tds, device,
                                       ctypes.byref(h)), "rt_scene_load_cli")
        return cls(h)

    def info(self) -> dict:
        v = np.zeros(len(INFO_NAMES), dtype=np.int64)
        _check(lib().rt_scene_info(self._h, v.ctypes.data, len(INFO_NAMES)), "rt_scene_info")
        return dict(zip(INFO_NAMES, v.tolist()))

    def save_name(self) -> str:
        """PNG name of the scene's `write` command (rt_scene_save_name)."""
        return _name_call(lib().rt_scene_save_name, self._h)

    def build_photons(self, seed: int):
        _check(lib().rt_photons_build(self._h, seed), "rt_photons_build")

    def build_photons_comm(self, comm, seed: int):
        """The photon pre-pass sharded over a communicator's ranks (rt_photons_build_comm; collective)."""
        _check(lib().rt_photons_build_comm(self._h, comm._h if comm is not None else None, seed),
               "rt_photons_build_comm")

    def shoot_photons(self, seed: int, first: int, count: int):
        """Photon shard [first, first+count) of every light -> (pos, pwr, per_light counts)."""
        nl = self.info()["lights"]
        per = np.zeros(max(1, nl), dtype=np.int64)
        _check(lib().rt_photons_shoot(self._h, seed, first, count, per.ctypes.data), "rt_photons_shoot")
        pos, pwr = self.photons()
        return pos, pwr, per[:nl]

    def set_photons(self, pos, pwr):
        pos = np.ascontiguousarray(pos, dtype=np.float64)
        pwr = np.ascontiguousarray(pwr, dtype=np.float64)
        _check(lib().rt_photons_set(self._h, pos.ctypes.data, pwr.ctypes.data, len(pos)), "rt_photons_set")

    def photon_map(self):
        """The device photon map: (nodes as raw uint8 [n_nodes, 128], root, ppos [n,3], ppwr [n,3])."""
        nn = ctypes.c_int64(0)
        root = ctypes.c_int32(0)
        _check(lib().rt_scene_photon_map(self._h, None, 0, None, None, 0, ctypes.byref(nn), ctypes.byref(root)),
               "rt_scene_photon_map")
        n = self.info()["photons"]
        nodes = np.zeros((nn.value, 128), dtype=np.uint8)
        ppos = np.zeros((n, 3)); ppwr = np.zeros((n, 3))
        _check(lib().rt_scene_photon_map(self._h, nodes.ctypes.data, nn.value, ppos.ctypes.data, ppwr.ctypes.data, n,
                                         ctypes.byref(nn), ctypes.byref(root)), "rt_scene_photon_map")
        return nodes, root.value, ppos, ppwr

    def photons(self):
        """(pos [n,3], pwr [n,3]) of the photon map in photon_list insertion order."""
        cnt = ctypes.c_int64(0)
        _check(lib().rt_scene_photons(self._h, None, None, 0, ctypes.byref(cnt)), "rt_scene_photons")
        n = cnt.value
        pos = np.zeros((n, 3)); pwr = np.zeros((n, 3))
        _check(lib().rt_scene_photons(self._h, pos.ctypes.data, pwr.ctypes.data, n, ctypes.byref(cnt)), "rt_scene_photons")
        return pos, pwr

    def render(self, W, H, spp=0, seed=0x5EED0001, rows=None, row_step=1, flags=0, row_band=1):
        p = params(W, H, spp, seed, rows, row_step, flags, row_band)
        n = nrows_of(p)
        rgb = np.zeros((n, W, 3), dtype=np.float32)
        argb = np.zeros((n, W), dtype=np.int32)
        _check(lib().rt_render(self._h, ctypes.byref(p), rgb.ctypes.data, argb.ctypes.data), "rt_render")
        return rgb, argb

    def render_argb_into(self, argb, W, H, spp=0, seed=0x5EED0001, flags=0):
        """The JNI draw() call: rt_render of the whole frame into a caller-owned
        host ARGB buffer (rndrdImg.pixels), no float plane; blocks until the pixels are there."""
        p = params(W, H, spp, seed, None, 1, flags, 1)
        assert argb.shape == (H, W) and argb.dtype == np.int32 and argb.flags.c_contiguous
        _check(lib().rt_render(self._h, ctypes.byref(p), None, argb.ctypes.data), "rt_render")

    def refine_steps(self, W, H) -> list[int]:
        """The `refine on` pass steps of a W x H render (myScene.setRefine); [1] without refine."""
        buf = np.zeros(16, dtype=np.int32)
        n = lib().rt_refine_steps(self._h, W, H, buf.ctypes.data, 16)
        if n < 0:
            raise RTError(f"rt_refine_steps: {lib().rt_last_error().decode()}")
        return buf[:n].tolist()

    def render_pass(self, W, H, step, skip_origin, rgb, argb, spp=0, seed=0x5EED0001, flags=0):
        """One refine pass into full-size host buffers rgb [H, W, 3] float32 / argb [H, W] int32 (in place)."""
        p = params(W, H, spp, seed, None, 1, flags, 1)
        assert rgb.shape == (H, W, 3) and rgb.dtype == np.float32 and rgb.flags.c_contiguous
        assert argb.shape == (H, W) and argb.dtype == np.int32 and argb.flags.c_contiguous
        _check(lib().rt_render_pass(self._h, ctypes.byref(p), step, int(bool(skip_origin)), rgb.ctypes.data,
                                    argb.ctypes.data), "rt_render_pass")

    def render_count(self, W, H, spp=0, seed=0x5EED0001, rows=None, row_step=1, row_band=1, flags=0):
        p = params(W, H, spp, seed, rows, row_step, flags, row_band)
        n = nrows_of(p)
        rgb = np.zeros((n, W, 3), dtype=np.float32)
        argb = np.zeros((n, W), dtype=np.int32)
        st = np.zeros(RT_ST_N, dtype=np.uint64)
        _check(lib().rt_render_count(self._h, ctypes.byref(p), rgb.ctypes.data, argb.ctypes.data, st.ctypes.data),
               "rt_render_count")
        return rgb, argb, dict(zip(ST_NAMES, st[: len(ST_NAMES)].tolist()))

    def variant(self, flags: int = 0) -> tuple[int, int]:
        """(timed, counted) feature masks F of the render_kernel<CNT, F> instantiations (rt_render_variant)."""
        a, b = ctypes.c_uint32(0), ctypes.c_uint32(0)
        _check(lib().rt_render_variant(self._h, flags, ctypes.byref(a), ctypes.byref(b)), "rt_render_variant")
        return a.value, b.value

    def render_device(self, p: RenderParams, rgb_ptr: int, argb_ptr: int, stream: int = 0):
        """Asynchronous render into device buffers (e.g. torch tensors' data_ptr()) on a HIP stream."""
        _check(lib().rt_render_device(self._h, ctypes.byref(p), ctypes.c_void_p(rgb_ptr), ctypes.c_void_p(argb_ptr),
                                      ctypes.c_void_p(stream)), "rt_render_device")

    def tile_layout(self, p: RenderParams) -> tuple[int, int, int, int]:
        """(ntiles, tiles_x, tw, th) of a render layout (rt_tile_layout)."""
        out = np.zeros(4, dtype=np.int32)
        _check(lib().rt_tile_layout(self._h, ctypes.byref(p), out.ctypes.data), "rt_tile_layout")
        return tuple(int(x) for x in out)

    def tile_costs(self, p: RenderParams) -> np.ndarray:
        """Measured wave time of every tile of the layout (uint32 [ntiles]; calibrates if needed)."""
        n = self.tile_layout(p)[0]
        c = np.zeros(n, dtype=np.uint32)
        r = lib().rt_tile_costs(self._h, ctypes.byref(p), c.ctypes.data, n)
        if r < 0:
            raise RTError(f"rt_tile_costs failed ({r}): {lib().rt_last_error().decode()}")
        return c

    def render_tiles_device(self, p: RenderParams, tiles: np.ndarray, rgb_ptr: int, argb_ptr: int, stream: int = 0):
        """Asynchronous render of the listed tiles (host int32 list) into whole-layout device buffers."""
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        _check(lib().rt_render_tiles_device(self._h, ctypes.byref(p), t.ctypes.data, len(t), ctypes.c_void_p(rgb_ptr),
                                            ctypes.c_void_p(argb_ptr), ctypes.c_void_p(stream)), "rt_render_tiles_device")

    def photon_kdtree(self) -> np.ndarray:
        """The device's copy of the reference's kd-tree: int32 [n, 4] (leaf-order photon, axis, left, right)."""
        n = self.info()["photons"]
        out = np.zeros((n, 4), dtype=np.int32)
        _check(lib().rt_scene_photon_kdtree(self._h, out.ctypes.data, n), "rt_scene_photon_kdtree")
        return out

    def photon_gather(self, pts) -> np.ndarray:
        """The render kernel's photon gather at points pts [n, 3] -> irradiance [n, 3] (rt_photon_gather)."""
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 3)
        out = np.zeros_like(pts)
        _check(lib().rt_photon_gather(self._h, pts.ctypes.data, out.ctypes.data, len(pts)), "rt_photon_gather")
        return out

    def render_pixels_device(self, p: RenderParams, pixels: np.ndarray, rgb_ptr: int, argb_ptr: int, stream: int = 0):
        """Asynchronous one-sample-per-wave render of the listed pixels (host int32 list) into whole-frame buffers."""
        t = np.ascontiguousarray(pixels, dtype=np.int32)
        _check(lib().rt_render_pixels_device(self._h, ctypes.byref(p), t.ctypes.data, len(t), ctypes.c_void_p(rgb_ptr),
                                             ctypes.c_void_p(argb_ptr), ctypes.c_void_p(stream)), "rt_render_pixels_device")

    def render_tiles_count(self, p: RenderParams, tiles: np.ndarray) -> dict:
        """Counters (rt_render_count's) of an instrumented render of the listed tiles only."""
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        st = np.zeros(RT_ST_N, dtype=np.uint64)
        _check(lib().rt_render_tiles_count(self._h, ctypes.byref(p), t.ctypes.data, len(t), st.ctypes.data),
               "rt_render_tiles_count")
        return dict(zip(ST_NAMES, st[: len(ST_NAMES)].tolist()))

    def time_render(self, W, H, spp=0, seed=0x5EED0001, rows=None, row_step=1, warmup=1, iters=3, flags=0,
                    row_band=1) -> float:
        p = params(W, H, spp, seed, rows, row_step, flags, row_band)
        ms = ctypes.c_double(0)
        _check(lib().rt_time_render(self._h, ctypes.byref(p), warmup, iters, ctypes.byref(ms)), "rt_time_render")
        return ms.value

    def close(self):
        if self._h:
            lib().rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# NodeD (csrc/rt_types.h): one 64-B line per child
NODE_DTYPE = np.dtype([("lmin", "<f8", 3), ("lmax", "<f8", 3), ("left", "<i4"), ("pad", "<i4", 3),
                       ("rmin", "<f8", 3), ("rmax", "<f8", 3), ("right", "<i4"), ("padR", "<i4", 3)])
assert NODE_DTYPE.itemsize == 128


def photon_maps_equal(a, b) -> bool:
    """Two Scene.photon_map() results are the same structure: refs / ranges / counts and the
    leaf-ordered photons bit-equal, boxes equal as numbers (a zero bound may carry either sign)."""
    na, ra, pa, wa = a
    nb, rb, pb, wb = b
    if na.shape != nb.shape or ra != rb:
        return False
    x, y = na.view(NODE_DTYPE).ravel(), nb.view(NODE_DTYPE).ravel()
    ints = all(np.array_equal(x[f], y[f]) for f in ("left", "pad", "right", "padR"))
    boxes = all(np.array_equal(x[f], y[f]) for f in ("lmin", "lmax", "rmin", "rmax"))
    return ints and boxes and np.array_equal(pa.view(np.uint64), pb.view(np.uint64)) and \
        np.array_equal(wa.view(np.uint64), wb.view(np.uint64))


def argb_to_rgb8(argb: np.ndarray) -> np.ndarray:
    a = argb.view(np.uint32)
    return np.stack([(a >> 16) & 255, (a >> 8) & 255, a & 255], -1).astype(np.uint8)
