"""The desc-driven boundary (VERDICT r01 Next #8): a scene built by hand as the JNI
`nativeCreate` would flatten it (myScene.java:1182,1481-1531) and handed to
rt_scene_create must render exactly like the same scene through rt_scene_load_cli.

CPU: the ctypes mirror (distraytracer_old_amd/desc.py) has the C compiler's layout for every
struct of include/distraytracer.h. GPU: c3shinyBall (two ground triangles, the mirror
sphere, three point lights, `diffuse` and `shiny` shaders) and a bvh_list of triangles."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from distraytracer_old_amd import desc, scenes

REPO = Path(__file__).resolve().parent.parent


def test_ctypes_layout_matches_c_header(tmp_path):
    import ctypes
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "distraytracer.h"', 'int main(void) {']
    for cname, T in desc.STRUCTS.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in T._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(REPO / "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                          check=True).stdout.splitlines())
    for cname, T in desc.STRUCTS.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(T), cname
        for f, _ in T._fields_:
            assert int(got[f"{cname} {f}"]) == getattr(T, f).offset, (cname, f)


def shiny_ball_desc():
    """data/c3shinyBall.cli, flattened by hand (myRTFileReader / myScene semantics)."""
    b = desc.SceneBuilder(fov=60, background=(0.2, 0.2, 1), rays_per_pixel=1)
    b.point_light((3, 4, 0), (.8, .2, .2))
    b.point_light((-3, 4, 0), (.2, .8, .2))
    b.point_light((0, 4, -5), (.2, .2, .8))
    ground = b.material(diffuse=(.8, .8, .8), ambient=(.2, .2, .2))  # diffuse .8 .8 .8 .2 .2 .2
    b.triangle([(-100, -1, -100), (100, -1, 100), (100, -1, -100)], ground)
    b.triangle([(100, -1, 100), (-100, -1, -100), (-100, -1, 100)], ground)
    ball = b.material(diffuse=(.8, .8, .8), ambient=(.2, .2, .2), phong=20, k_refl=1)  # shiny ... 20 1 0 0
    b.sphere(1, (0, 0.5, -3), ball)
    return b


@pytest.mark.gpu
def test_desc_scene_renders_like_cli_scene():
    from distraytracer_old_amd import rt
    b = shiny_ball_desc()
    with desc.scene_from_desc(b.desc()) as g:
        info = g.info()
        assert (info["objects"], info["lights"]) == (3, 3)
        rgb_d, argb_d = g.render(160, 160, spp=4, seed=7)
        _, kat = g.render(300, 300, spp=1, rows=(150, 151))
    with rt.Scene.load_cli("c3shinyBall.cli", textures={}) as c:
        rgb_c, argb_c = c.render(160, 160, spp=4, seed=7)
    assert np.array_equal(argb_d, argb_c)
    assert np.array_equal(rgb_d.view(np.uint32), rgb_c.view(np.uint32))
    assert (int(kat[0, 150]) & 0xFFFFFFFF) == 0xFFFFFFA9  # SURVEY 8(c) KAT


@pytest.mark.gpu
def test_desc_bvh_group_renders_like_cli_scene():
    """begin_list / read bun500 / end_accel as accel members + an rt_accel_desc with its CTM."""
    from distraytracer_old_amd import rt
    tris = scenes._parse_tris(scenes.SCENE_DIR / "bun500.cli")
    # the .cli equivalent: written next to the scenes so both paths see the same triangles
    b = desc.SceneBuilder(fov=60, background=(0.1, 0.1, 0.1), rays_per_pixel=1)
    b.point_light((2, 4, 2), (.9, .9, .9))
    m = b.material(diffuse=(.7, .5, .3), ambient=(.1, .1, .1), phong=10, k_refl=.2)
    first = len(b.members)
    ctm = (.5, 0, 0, 0, 0, .5, 0, 0, 0, 0, .5, -3, 0, 0, 0, 1)  # translate 0 0 -3, scale .5
    for t in desc.np_tris(tris):
        b.triangle(t, m, ctm=ctm, in_list=True)
    b.end_accel(first, bvh=True, ctm=ctm)
    with desc.scene_from_desc(b.desc()) as g:
        info = g.info()
        rgb_d, argb_d = g.render(128, 128, spp=2, seed=3)
    with rt.Scene.load_cli("desc_bun500.cli", textures={}) as c:
        ic = c.info()
        rgb_c, argb_c = c.render(128, 128, spp=2, seed=3)
    assert info["bvh_internal"] == ic["bvh_internal"] and info["bvh_leaves"] == ic["bvh_leaves"]
    assert np.array_equal(argb_d, argb_c)
    assert np.array_equal(rgb_d.view(np.uint32), rgb_c.view(np.uint32))
