"""ctypes mirror of the scene description structs of include/distraytracer.h.

This is what a host that keeps its own scene parser -- the reference's Java `myScene`
through JNI (INTEGRATION.md `nativeCreate`), or Python -- fills in and hands to
`rt_scene_create`: the flattened `objList` / `lightList` / shaders / CTMs / accel groups
that `myFOVScene.draw()` reads (myScene.java:1182,1481-1531). Field meanings follow the
header; `tests/test_desc.py` checks the layout against the C compiler's and renders a
hand-built desc.
"""
from __future__ import annotations

import ctypes

import numpy as np

D16 = ctypes.c_double * 16
D3 = ctypes.c_double * 3

PRIM_TRIANGLE, PRIM_QUAD, PRIM_PLANE, PRIM_SPHERE, PRIM_MOVING_SPHERE, PRIM_CYLINDER, PRIM_HOLLOW_CYLINDER, PRIM_BOX = range(8)
LIGHT_POINT, LIGHT_SPOT, LIGHT_DISK = range(3)
CAMERA_FOV, CAMERA_FISHEYE, CAMERA_ORTHO = range(3)
REF_INSTANCE = 0x40000000
IDENTITY = (1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1)


class PrimDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("material", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("nverts", ctypes.c_int32), ("ctm", D16), ("v", (ctypes.c_double * 3) * 4),
                ("uv", (ctypes.c_double * 2) * 4), ("p", ctypes.c_double * 12)]


class MaterialDesc(ctypes.Structure):
    _fields_ = [("simple", ctypes.c_int32), ("texture", ctypes.c_int32), ("tex_top", ctypes.c_int32),
                ("use_photon_map", ctypes.c_int32), ("caustic_photons", ctypes.c_int32), ("octaves", ctypes.c_int32),
                ("rnd_colors", ctypes.c_int32), ("use_fwd_trans", ctypes.c_int32),
                ("diffuse", D3), ("ambient", D3), ("specular", D3),
                ("phong_exp", ctypes.c_double), ("k_refl", ctypes.c_double), ("k_refl_clr", D3),
                ("k_trans", ctypes.c_double), ("perm", ctypes.c_double), ("perm_clr", D3),
                ("noise_scale", ctypes.c_double), ("turb_mult", ctypes.c_double), ("color_scale", ctypes.c_double),
                ("color_mult", ctypes.c_double), ("period_mult", D3), ("colors", D3 * 16),
                ("num_colors", ctypes.c_int32), ("dist_func", ctypes.c_int32), ("roi_func", ctypes.c_int32),
                ("num_pts_dist", ctypes.c_int32), ("avg_per_cell", ctypes.c_double), ("mortar_thresh", ctypes.c_double)]


class LightDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("pad", ctypes.c_int32), ("pos", D3), ("color", D3), ("dir", D3),
                ("inner_deg", ctypes.c_double), ("outer_deg", ctypes.c_double), ("radius", ctypes.c_double),
                ("ctm", D16)]


class AccelDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("first", ctypes.c_int32), ("count", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("ctm", D16)]


class InstanceDesc(ctypes.Structure):
    _fields_ = [("base", ctypes.c_int32), ("material", ctypes.c_int32), ("ctm", D16), ("origin", D3)]


class TextureDesc(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int32), ("h", ctypes.c_int32), ("rgb", ctypes.c_void_p)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("num_prims", ctypes.c_int32), ("prims", ctypes.POINTER(PrimDesc)),
                ("num_materials", ctypes.c_int32), ("materials", ctypes.POINTER(MaterialDesc)),
                ("num_lights", ctypes.c_int32), ("lights", ctypes.POINTER(LightDesc)),
                ("num_accels", ctypes.c_int32), ("accels", ctypes.POINTER(AccelDesc)),
                ("accel_members", ctypes.POINTER(ctypes.c_int32)),
                ("num_top", ctypes.c_int32), ("top", ctypes.POINTER(ctypes.c_int32)),
                ("num_textures", ctypes.c_int32), ("textures", ctypes.POINTER(TextureDesc)),
                ("fov", ctypes.c_double), ("background", D3), ("bkg_texture", ctypes.c_int32),
                ("rays_per_pixel", ctypes.c_int32), ("skydome", ctypes.c_double * 4), ("dof", ctypes.c_int32),
                ("camera", ctypes.c_int32), ("lens_radius", ctypes.c_double), ("lens_focal", ctypes.c_double),
                ("photon_mode", ctypes.c_int32), ("photon_count", ctypes.c_int32), ("photon_k", ctypes.c_int32),
                ("pad1", ctypes.c_int32), ("photon_max_dist", ctypes.c_double), ("camera_param", ctypes.c_double * 2),
                ("num_instances", ctypes.c_int32), ("pad2", ctypes.c_int32),
                ("instances", ctypes.POINTER(InstanceDesc))]


STRUCTS = {"rt_prim_desc": PrimDesc, "rt_material_desc": MaterialDesc, "rt_light_desc": LightDesc,
           "rt_accel_desc": AccelDesc, "rt_instance_desc": InstanceDesc, "rt_texture_desc": TextureDesc,
           "rt_scene_desc": SceneDesc}


class SceneBuilder:
    """Accumulates a flattened scene the way a `myScene` walk would (objList order = creation
    order of top-level objects, one material per object) and produces an rt_scene_desc.
    Keeps every array alive for as long as the builder lives."""

    def __init__(self, fov=60.0, background=(0, 0, 0), rays_per_pixel=1):
        self.prims, self.mats, self.lights, self.accels, self.members, self.top = [], [], [], [], [], []
        self.insts, self.textures, self._keep = [], [], []
        self.fov, self.background, self.rpp = fov, background, rays_per_pixel

    def material(self, diffuse=(0, 0, 0), ambient=(0, 0, 0), specular=(0, 0, 0), phong=0.0, k_refl=0.0,
                 k_trans=0.0, perm=0.0, perm_clr=None, simple=False) -> int:
        """myObjShader.setCurrColors state (colours already clamped <= 1, as myColor does)."""
        m = MaterialDesc()
        m.simple = int(simple)
        m.tex_top = -1
        for name, c in (("diffuse", diffuse), ("ambient", ambient), ("specular", specular)):
            getattr(m, name)[:] = [min(1.0, x) for x in c]
        m.phong_exp, m.k_refl, m.k_trans, m.perm = phong, k_refl, k_trans, perm
        m.k_refl_clr[:] = [min(1.0, k_refl)] * 3
        m.perm_clr[:] = [min(1.0, x) for x in (perm_clr if perm_clr is not None else (perm,) * 3)]
        self.mats.append(m)
        return len(self.mats) - 1

    def _prim(self, typ, mat, ctm):
        p = PrimDesc()
        p.type, p.material = typ, mat
        p.ctm[:] = ctm
        return p

    def _add(self, p, in_list):
        self.prims.append(p)
        idx = len(self.prims) - 1
        (self.members if in_list else self.top).append(idx)
        return idx

    def triangle(self, v, mat, ctm=IDENTITY, in_list=False):
        p = self._prim(PRIM_TRIANGLE, mat, ctm)
        p.nverts = 3
        for i in range(3):
            p.v[i][:] = v[i]
        return self._add(p, in_list)

    def sphere(self, radius, center, mat, ctm=IDENTITY, in_list=False):
        p = self._prim(PRIM_SPHERE, mat, ctm)
        p.p[0:3] = center
        p.p[3:6] = [radius] * 3
        return self._add(p, in_list)

    def end_accel(self, first_member, bvh=True, ctm=IDENTITY):
        """begin_list ... end_accel (bvh) / end_list over members [first_member, len(members))."""
        a = AccelDesc()
        a.type, a.first, a.count = int(bvh), first_member, len(self.members) - first_member
        a.ctm[:] = ctm
        self.accels.append(a)
        self.top.append(~(len(self.accels) - 1))

    def point_light(self, pos, color, ctm=IDENTITY):
        L = LightDesc()
        L.type = LIGHT_POINT
        L.pos[:] = pos
        L.color[:] = [min(1.0, x) for x in color]
        L.ctm[:] = ctm
        self.lights.append(L)

    def desc(self) -> SceneDesc:
        def arr(T, xs):
            a = (T * max(1, len(xs)))(*xs)
            self._keep.append(a)
            return a

        d = SceneDesc()
        d.num_prims, d.prims = len(self.prims), arr(PrimDesc, self.prims)
        d.num_materials, d.materials = len(self.mats), arr(MaterialDesc, self.mats)
        d.num_lights, d.lights = len(self.lights), arr(LightDesc, self.lights)
        d.num_accels, d.accels = len(self.accels), arr(AccelDesc, self.accels)
        d.accel_members = arr(ctypes.c_int32, self.members)
        d.num_top, d.top = len(self.top), arr(ctypes.c_int32, self.top)
        d.num_textures, d.textures = 0, arr(TextureDesc, [])
        d.fov = self.fov
        d.background[:] = [min(1.0, x) for x in self.background]
        d.bkg_texture = -1
        d.rays_per_pixel = self.rpp
        d.camera = CAMERA_FOV
        d.num_instances, d.instances = 0, arr(InstanceDesc, [])
        self._keep.append(d)
        return d


def scene_from_desc(desc: SceneDesc, device: int = 0):
    """rt_scene_create(desc, device) -> rt.Scene."""
    from . import rt

    L = rt.lib()
    h = ctypes.c_void_p()
    rc = L.rt_scene_create(ctypes.byref(desc), device, ctypes.byref(h))
    if rc != 0:
        raise rt.RTError(f"rt_scene_create failed ({rc}): {L.rt_last_error().decode()}")
    return rt.Scene(h)


def np_tris(tris: np.ndarray):
    """[n, 3, 3] float64 -> list of vertex triples (tuples) for SceneBuilder.triangle."""
    return [tuple(map(tuple, t)) for t in np.asarray(tris, dtype=np.float64)]
