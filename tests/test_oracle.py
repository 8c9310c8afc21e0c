"""Oracle (CPU restatement) pinned by the hand-derived known-answer pixels of
SURVEY.md 8(c) / BASELINE.md 6 and by the reference BVH topology (SURVEY 8(d) C3,
Appendix A Q1). No GPU needed."""
import numpy as np
import pytest

from distraytracer_old_amd import scenes
from oracle.oracle import OracleScene


def _px(cli, W, H, row, col, spp=1):
    o = OracleScene(scenes.SCENE_DIR, cli, scenes.prepare(cli))
    rgb, argb, _ = o.render(W, H, spp=spp, rows=(row, row + 1))
    return rgb[0, col], int(argb[0, col]) & 0xFFFFFFFF


def test_kat_t01_300():
    rgb, argb = _px("t01.cli", 300, 300, 150, 150)
    np.testing.assert_allclose(rgb, [0.2 + 0.5 * 8 / np.sqrt(90), 0, 0], atol=1e-6)
    assert argb == 0xFF9E0000


def test_kat_t01_256_centre_is_same_axis_ray():
    rgb, argb = _px("t01.cli", 256, 256, 128, 128)
    assert argb == 0xFF9E0000


def test_kat_c3shinyball_300():
    rgb, argb = _px("c3shinyBall.cli", 300, 300, 150, 150)
    np.testing.assert_allclose(rgb, [1.0, 1.0, 0.665113], atol=2e-6)
    assert argb == 0xFFFFFFA9


def test_bvh_topology_c3():
    """69,451 synthetic triangles -> 69,450 kept (Q1), 16,383 internal / 16,384 leaves, depth 14."""
    o = OracleScene(scenes.SCENE_DIR, "c3_bun69k.cli", scenes.prepare("c3_bun69k.cli"))
    i = o.info()
    assert (i["bvh_internal"], i["bvh_leaves"], i["bvh_depth"], i["bvh_prims"]) == (16383, 16384, 14, 69450)
    assert i["prims"] == 69453 and i["objects"] == 3 and i["lights"] == 2


def test_oracle_deterministic_and_row_decomposable():
    o = OracleScene(scenes.SCENE_DIR, "c3shinyBall.cli", scenes.prepare("c3shinyBall.cli"))
    a = o.render(64, 64, spp=3, seed=7)
    b = o.render(64, 64, spp=3, seed=7, threads=1)
    assert np.array_equal(a[1], b[1])
    c = o.render(64, 64, spp=3, seed=7, rows=(1, 64), row_step=4)
    assert np.array_equal(c[1], a[1][1::4])


def test_seed_changes_stochastic_pixels_only():
    o = OracleScene(scenes.SCENE_DIR, "p2_t05.cli", scenes.prepare("p2_t05.cli"))
    a = o.render(48, 48, spp=4, seed=1)[0]
    b = o.render(48, 48, spp=4, seed=2)[0]
    assert not np.array_equal(a, b)
    assert abs(float(a.mean()) - float(b.mean())) < 0.02


def test_photon_map_builds_kdtree():
    """t11 diffuse photons with a reduced photon count (the full 1e6/light runs on the GPU path)."""
    import shutil
    import tempfile
    from pathlib import Path

    d = Path(tempfile.mkdtemp())
    src = (scenes.SCENE_DIR / "t11.cli").read_text().replace("diffuse_photons  1000000  200 0.1",
                                                             "diffuse_photons  20000  50 0.1")
    (d / "t11s.cli").write_text(src)
    try:
        o = OracleScene(d, "t11s.cli")
        n = o.build_photons(0x5EED0005)
        assert 5000 < n < 80000
        rgb, argb, st = o.render(32, 32, spp=1, seed=0x5EED0005)
        assert st["photon"] > 0 and np.isfinite(rgb).all()
    finally:
        shutil.rmtree(d)


def test_kat_ortho_and_fisheye_centre():
    """Hand-derived KAT (myOrthoScene / myFishEyeScene, myScene.java:1535-1755): the centre
    pixel's ray runs down -z in both old_t07 (ortho 6 6, origin (0,0,0)) and old_t10 (fisheye
    180: r = 0 -> theta = 0 -> d = (0,0,-1)); it hits the unit sphere at (0,0,-6) in
    P = (0,0,-5), N = (0,0,1); light (0,0,0) .2 gives .8*.2*1, light (4,4,0) 1 gives
    .8*(N.L = 5/sqrt(57)); ambient 0 -> 0.16 + 0.8*5/sqrt(57) = 0.689813 -> 0xFFAFAFAF.
    A fisheye pixel outside the image circle is blkColor (0xFF000000)."""
    expect = 0.16 + 0.8 * 5 / np.sqrt(57)
    for cli in ("old_t07.cli", "old_t10.cli"):
        o = OracleScene(scenes.SCENE_DIR, cli, {})
        rgb, argb, _ = o.render(300, 300, spp=1, rows=(150, 151))
        assert np.allclose(rgb[0, 150], expect, atol=1e-6)
        assert (int(argb[0, 150]) & 0xFFFFFFFF) == 0xFFAFAFAF
    o = OracleScene(scenes.SCENE_DIR, "old_t10.cli", {})
    _, argb, st = o.render(300, 300, spp=1, rows=(0, 1))
    assert (int(argb[0, 0]) & 0xFFFFFFFF) == 0xFF000000
    assert st["camera"] < 300  # corners of the top row lie outside the circle and trace nothing
