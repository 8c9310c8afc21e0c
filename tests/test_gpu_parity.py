"""GPU parity: the HIP trace loop (through the C ABI) vs the oracle on the same
seeded inputs, at sizes the oracle finishes in seconds; plus size-independent
properties at BASELINE.json's full C3 size.

Tolerance: per-channel |d| <= 1e-4 (tests/parity.py); decision mismatches
(pixels beyond it) are counted and bounded per test.
"""
import numpy as np
import pytest

from distraytracer_old_amd import rt, scenes
from oracle.oracle import OracleScene
from tests.parity import assert_exact_decisions, compare

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001


def both(cli, W, H, spp, seed=SEED, rows=None):
    tex = scenes.prepare(cli)
    g = rt.Scene.load_cli(cli, textures=tex)
    o = OracleScene(scenes.SCENE_DIR, cli, tex)
    rg, ag = g.render(W, H, spp=spp, seed=seed, rows=rows)
    ro, ao, _ = o.render(W, H, spp=spp, seed=seed, rows=rows)
    return g, o, (rg, ag), (ro, ao)


def test_c1_t01_kat_and_parity():
    g, o, (rg, ag), (ro, ao) = both("t01.cli", 256, 256, 1)
    assert (int(ag[128, 128]) & 0xFFFFFFFF) == 0xFF9E0000
    assert abs(rg[128, 128, 0] - 0.621637) < 1e-6
    c = compare(rg, ag, ro, ao)
    assert c["mismatch"] == 0, c
    assert c["argb_mismatch_on_good"] == 0, c


def test_c2_shiny_ball_kat_and_parity():
    g, o, (rg, ag), (ro, ao) = both("c3shinyBall.cli", 512, 512, 1)
    c = compare(rg, ag, ro, ao)
    assert c["mismatch"] == 0, c
    assert c["argb_mismatch_on_good"] == 0, c
    r300, a300 = g.render(300, 300, spp=1, rows=(150, 151))
    assert (int(a300[0, 150]) & 0xFFFFFFFF) == 0xFFFFFFA9
    np.testing.assert_allclose(r300[0, 150], [1.0, 1.0, 0.665113], atol=2e-6)


def test_c3_bun69k_small_parity():
    g, o, (rg, ag), (ro, ao) = both("c3_bun69k.cli", 256, 256, 4)
    assert_exact_decisions(compare(rg, ag, ro, ao))


def test_c4_planets_small_parity():
    g, o, (rg, ag), (ro, ao) = both("plnts3ColsBunnies.cli", 160, 160, 2, seed=0x5EED0004)
    assert_exact_decisions(compare(rg, ag, ro, ao))


@pytest.mark.parametrize("cli,spp", [("old_t07.cli", 1), ("old_t07.cli", 4), ("old_t10.cli", 1), ("old_t10.cli", 4),
                                     ("planets3Ortho.cli", 2)])
def test_camera_scenes_parity(cli, spp):
    """orthographic (old_t07, planets3Ortho: textures + glass) and fisheye 180 (old_t10) cameras
    (myOrthoScene / myFishEyeScene, myScene.java:1535-1755), 1 spp and jittered."""
    g, o, (rg, ag), (ro, ao) = both(cli, 96, 96, spp)
    assert_exact_decisions(compare(rg, ag, ro, ao))
    if cli == "old_t10.cli" and spp == 1:  # outside the image circle: blkColor
        assert (int(ag[0, 0]) & 0xFFFFFFFF) == 0xFF000000 and rg[0, 0].max() == 0


@pytest.mark.parametrize("cli,spp", [("p2_t05.cli", 4), ("p2_t07.cli", 4), ("c2clear.cli", 1), ("p2_t03.cli", 4),
                                     ("p3_t09.cli", 2), ("p4_t05.cli", 2), ("p4_t06_2.cli", 2)])
def test_feature_scenes_parity(cli, spp):
    """disk light (p2_t05), depth of field (p2_t07), refraction (c2clear), motion blur (p2_t03),
    procedural wood (p3_t09 = C3 with its wood line; myBaseWoodTexture), wood2 with named
    noise_color (p4_t05; myWoodTexture) and marble with custom noise_color (p4_t06_2)."""
    g, o, (rg, ag), (ro, ao) = both(cli, 128, 128, spp)
    assert_exact_decisions(compare(rg, ag, ro, ao))


@pytest.mark.parametrize("cli", [f"p4_st0{i}.cli" for i in range(1, 10)])
def test_stone_parity(cli):
    """cellular `stone` texture (myCellularTexture, myTextureHandler.java:380-498): st01-st07 walk
    the ROI functions 2..8 with Euclid distance, st08 nearestROI with Manhattan distance,
    st09 altExpROI; all read worleyClrs.cli (10 noise colours)."""
    g, o, (rg, ag), (ro, ao) = both(cli, 96, 96, 1)
    assert_exact_decisions(compare(rg, ag, ro, ao))


@pytest.mark.parametrize("cli,spp", [("p3_t01.cli", 1), ("p3_t02.cli", 2), ("p3_t03.cli", 1), ("p4_t02.cli", 1),
                                     ("p4_t05Alt.cli", 1), ("p3_t10.cli", 1), ("p3_t11.cli", 2),
                                     ("p3_t02_sierp.cli", 1), ("p3_t11_sierp.cli", 1)])
def test_instance_parity(cli, spp):
    """named_object / instance (myInstance, mySceneObject.java:95-145): instanced spheres
    (p3_t01-03, scaled), textured (p4_t02, p4_t05Alt), instanced bun69k BVHs with instance
    shaders (p3_t10, p3_t11: hits stay in the named BVH's space, Q4), and sierpinski BVHs of
    instances (p3_t02_sierp: 341 spheres; p3_t11_sierp: 21,845 bun69k instances, two-level)."""
    scenes.ensure_bun69k()
    g, o, (rg, ag), (ro, ao) = both(cli, 96, 96, spp)
    assert_exact_decisions(compare(rg, ag, ro, ao))


def test_c3_full_size_properties():
    """BASELINE C3 size (1024^2, 16 spp): deterministic, band-decomposable, and
    matching the oracle on a row subsample."""
    tex = scenes.prepare("c3_bun69k.cli")
    g = rt.Scene.load_cli("c3_bun69k.cli", textures=tex)
    rg, ag = g.render(1024, 1024, spp=16, seed=SEED)
    rg2, ag2 = g.render(1024, 1024, spp=16, seed=SEED)
    assert np.array_equal(ag, ag2) and np.array_equal(rg, rg2)
    top, at = g.render(1024, 1024, spp=16, seed=SEED, rows=(0, 512))
    bot, ab = g.render(1024, 1024, spp=16, seed=SEED, rows=(512, 1024))
    assert np.array_equal(np.concatenate([at, ab]), ag)
    il, ail = g.render(1024, 1024, spp=16, seed=SEED, rows=(3, 1024), row_step=8)
    assert np.array_equal(ail, ag[3::8])
    o = OracleScene(scenes.SCENE_DIR, "c3_bun69k.cli", tex)
    ro, ao, _ = o.render(1024, 1024, spp=16, seed=SEED, rows=(5, 1024), row_step=64)
    assert_exact_decisions(compare(rg[5::64], ag[5::64], ro, ao))
    assert rg.min() >= 0 and rg.max() <= 1.0


@pytest.mark.parametrize("cli,W,spp", [("c3_bun69k.cli", 128, 2), ("plnts3ColsBunnies.cli", 48, 2)])
def test_ray_counts_match_oracle(cli, W, spp):
    """The instrumented kernel counts the reference algorithm's work exactly when nothing is
    culled (RT_RENDER_NOCULL): rays, triangle / quad / implicit tests, lights, texels. (Box
    tests are counted per node visit on the GPU and per test call in the oracle: not compared.)"""
    tex = scenes.prepare(cli)
    g = rt.Scene.load_cli(cli, textures=tex)
    _, _, sg = g.render_count(W, W, spp=spp, seed=SEED, flags=rt.RENDER_NOCULL)
    o = OracleScene(scenes.SCENE_DIR, cli, tex)
    _, _, so = o.render(W, W, spp=spp, seed=SEED)
    so = dict(so, implicit=so["sphere"])
    for k in ("camera", "shadow", "refl", "refr", "tri", "quad", "implicit", "light", "texel"):
        assert sg[k] == so[k], (k, sg[k], so[k])
    # per-wave record loads never exceed the per-lane ones; culling and the nearest-first order only
    # remove work (the counting kernel is the timed variant's instantiation, rt_render_variant)
    timed, counted = g.variant()
    assert timed == counted
    _, _, sc = g.render_count(W, W, spp=spp, seed=SEED)
    for k in ("node", "tri", "quad", "implicit", "light", "photon"):
        assert sc["w_" + k] <= sc[k], k
    for k in ("node", "tri", "quad", "implicit", "light", "photon"):
        assert sc[k] <= sg[k], k
    for k in ("camera", "shadow", "refl", "refr", "light", "texel"):
        assert sc[k] == sg[k], k


@pytest.mark.parametrize("mode,spec", [("diffuse", "diffuse_photons  20000  50 0.1"),
                                       ("caustic", "caustic_photons  20000  40 0.05")])
def test_photon_map_parity(tmp_path, mode, spec):
    """C5 path (t11 Cornell box) with a reduced photon count: GPU photon shooting + map + kNN
    gather vs the oracle. Emission / bounce / Fresnel trig is the shared fdlibm restatement
    (csrc/jfdlibm.h), so the photon_list is bit-identical and every decision agrees."""
    src = (scenes.SCENE_DIR / "t11.cli").read_text().replace("diffuse_photons  1000000  200 0.1", spec)
    (tmp_path / "t11s.cli").write_text(src)
    g = rt.Scene.load_cli("t11s.cli", scene_dir=tmp_path, textures={})
    o = OracleScene(tmp_path, "t11s.cli")
    seed = 0x5EED0005
    g.build_photons(seed)
    n_o = o.build_photons(seed)
    assert g.info()["photons"] == n_o
    gp, gw = g.photons()
    op, ow = o.photons()
    assert np.array_equal(gp.view(np.uint64), op.view(np.uint64))
    assert np.array_equal(gw.view(np.uint64), ow.view(np.uint64))
    rg, ag = g.render(64, 64, spp=2, seed=seed)
    ro, ao, _ = o.render(64, 64, spp=2, seed=seed)
    assert_exact_decisions(compare(rg, ag, ro, ao))


def test_c5_full_prepass_and_k200_gather_parity():
    """C5 at its real parameters (data/t11.cli unmodified: diffuse_photons 1000000 200 0.1,
    i.e. 2.68 M stored photons, k = 200, counting-window selection; myLight.java:389-445,
    myScene.java:1000-1091): the GPU pre-pass's photon_list equals the oracle's bit for bit,
    and the k = 200 gathers over that list agree on every pixel (64x64, 2 spp)."""
    seed = 0x5EED0005
    g = rt.Scene.load_cli("t11.cli", textures={})
    g.build_photons(seed)
    o = OracleScene(scenes.SCENE_DIR, "t11.cli")
    n_o = o.build_photons(seed)
    gp, gw = g.photons()
    op, ow = o.photons()
    assert len(gp) == n_o > 2_600_000
    assert np.array_equal(gp.view(np.uint64), op.view(np.uint64))
    assert np.array_equal(gw.view(np.uint64), ow.view(np.uint64))
    rg, ag = g.render(64, 64, spp=2, seed=seed)
    ro, ao, _ = o.render(64, 64, spp=2, seed=seed)
    assert_exact_decisions(compare(rg, ag, ro, ao))


def test_knn_u16_bucket_fallback_renders_identically(monkeypatch):
    """The kNN counting passes keep 128 u8 buckets per lane, repeat a pass with 64 u16 buckets for a
    lane whose u8 buckets may have carried, and with 16 u32 buckets for a lane with more photons
    bucketed than the u16 halves hold. DISTRAYTRACER_KNN_U16_MAX (read at scene creation) lowers both
    limits to 100 photons, so nearly every pass of C5's k = 200 gather takes both fallbacks: the
    image must not change."""
    seed = 0x5EED0005
    imgs = []
    for lim in (None, "100"):
        if lim:
            monkeypatch.setenv("DISTRAYTRACER_KNN_U16_MAX", lim)
        g = rt.Scene.load_cli("t11.cli", textures={})
        g.build_photons(seed)
        imgs.append(g.render(64, 64, spp=2, seed=seed))
    (r0, a0), (r1, a1) = imgs
    assert np.array_equal(a0, a1)
    assert np.array_equal(r0.view(np.uint32), r1.view(np.uint32))


@pytest.mark.parametrize("cli,W,spp", [("c3_bun69k.cli", 128, 2), ("t01.cli", 128, 1), ("p2_t05.cli", 96, 2),
                                       ("c2clear.cli", 96, 1), ("plnts3ColsBunnies.cli", 96, 1),
                                       ("t11.cli", 64, 1), ("p3_t11_sierp.cli", 64, 1)])
def test_specialised_kernel_equals_generic(cli, W, spp):
    """The feature-specialised kernel variant picked for a scene renders bit-identically
    to the all-features kernel (RT_RENDER_GENERIC)."""
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    rs, as_ = g.render(W, W, spp=spp, seed=SEED)
    rg, ag = g.render(W, W, spp=spp, seed=SEED, flags=rt.RENDER_GENERIC)
    assert np.array_equal(as_, ag)
    assert np.array_equal(rs.view(np.uint32), rg.view(np.uint32))


@pytest.mark.parametrize("cli,W,spp", [("plnts3ColsBunnies.cli", 96, 2), ("t11.cli", 64, 1), ("p2_t05.cli", 64, 2)])
def test_compacted_shadow_rays_oracle_parity(cli, W, spp):
    """RT_RENDER_SHCOMPACT against the oracle (not only against the default HIP path): C4's scene,
    the photon-map Cornell box and the disk light, in the scene's variant."""
    scenes.ensure_bun69k()
    tex = scenes.prepare(cli)
    g = rt.Scene.load_cli(cli, textures=tex)
    o = OracleScene(scenes.SCENE_DIR, cli, tex)
    if cli == "t11.cli":  # the same photon_list on both sides (test_c5_full_prepass_and_k200_gather_parity)
        g.build_photons(SEED)
        o.build_photons(SEED)
    rg, ag = g.render(W, W, spp=spp, seed=SEED, flags=rt.RENDER_SHCOMPACT)
    ro, ao, _ = o.render(W, W, spp=spp, seed=SEED)
    assert_exact_decisions(compare(rg, ag, ro, ao))


@pytest.mark.parametrize("cli,W,spp", [("c3_bun69k.cli", 128, 4), ("plnts3ColsBunnies.cli", 96, 4),
                                       ("p2_t05.cli", 96, 2), ("c3spotLight.cli", 96, 2), ("p2_t03.cli", 96, 2),
                                       ("c2clear.cli", 96, 1), ("t11.cli", 64, 1), ("p3_t11_sierp.cli", 64, 1)])
def test_compacted_shadow_rays_render_identically(cli, W, spp):
    """RT_RENDER_SHCOMPACT (the wave's shading steps in step, its (hit, light) shadow rays
    numbered by ballot + prefix count and traced one per lane): bit-identical to the lane-by-lane
    light loop -- point / spot / disk lights, moving spheres (keyed shadow-ray times), glass,
    photon map, instances -- in the scene's variant and the generic one."""
    scenes.ensure_bun69k()
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    ra, aa = g.render(W, W, spp=spp, seed=SEED)
    for flags in (rt.RENDER_SHCOMPACT, rt.RENDER_SHCOMPACT | rt.RENDER_GENERIC):
        rb, ab = g.render(W, W, spp=spp, seed=SEED, flags=flags)
        assert np.array_equal(aa, ab), flags
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32)), flags


@pytest.mark.parametrize("cli,W,spp", [("plnts3ColsBunnies.cli", 128, 4), ("p2_t03.cli", 96, 2),
                                       ("c3spotLight.cli", 96, 2), ("p2_t05.cli", 96, 2), ("c4.cli", 96, 2),
                                       ("cylinder1.cli", 96, 2)])
def test_wave_shadow_cull_renders_identically(cli, W, spp):
    """The wave-level shadow candidate test (SCENE_WAVE_CULL: an entry whose bounding sphere
    stays farther than the lanes' spread from the wave's first shadow segment is skipped) gives
    the image of the plain per-lane scan (RT_RENDER_NOWAVECULL) and of the reference's full scan
    (RT_RENDER_NOCULL) bit for bit: spot / point / disk lights, moving spheres, cylinders, glass."""
    scenes.ensure_bun69k()
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    ra, aa = g.render(W, W, spp=spp, seed=SEED)
    for flags in (rt.RENDER_NOWAVECULL, rt.RENDER_NOCULL):
        rb, ab = g.render(W, W, spp=spp, seed=SEED, flags=flags)
        assert np.array_equal(aa, ab), flags
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32)), flags


WAVE_CULL_SCENE = """fov 60
background 0.2 0.2 0.3
point_light 2 5 0 .6 .6 .6
spotlight -2 6 -2  0.3 -1 -0.2  15 40  .5 .5 .5
push
translate 0.5 1 -3
point_light 0 1 0 .3 .3 .3
pop
push
translate 0 -1 -4
rotate 20 0 1 0
rotate 10 1 0 0
scale 3 1 2
diffuse .7 .7 .7 .1 .1 .1
begin quad
vertex -1 0 -1
vertex 1 0 -1
vertex 1 0 1
vertex -1 0 1
end
pop
push
translate 0 0 -6
rotate 30 0 1 0
diffuse .3 .6 .3 .1 .1 .1
begin quad
vertex -2 -1 0
vertex 2 -1 0
vertex 2 2 0
vertex -2 2 0
end
pop
diffuse .8 .2 .2 .1 .1 .1
sphere .5 -0.8 -0.3 -3.5
push
scale 1 1.5 1
sphere .4 0.9 0.0 -3
pop
cyl .3 1  1.5 -1 -4.5
"""


def test_wave_shadow_cull_transformed_quads(tmp_path):
    """The wave-level cull's world planes (A^-T N, d - n.b of each quad's CTM) and bounding
    spheres under rotated / scaled CTMs, a light under a translation (not eligible when its CTM
    applies), point and spot lights: bit-identical to the per-lane scan and to the full scan."""
    (tmp_path / "wc.cli").write_text(WAVE_CULL_SCENE)
    g = rt.Scene.load_cli("wc.cli", scene_dir=tmp_path, textures={})
    ra, aa = g.render(96, 96, spp=4, seed=SEED)
    assert len(np.unique(aa)) > 50  # lit, shadowed and background pixels
    for flags in (rt.RENDER_NOWAVECULL, rt.RENDER_NOCULL):
        rb, ab = g.render(96, 96, spp=4, seed=SEED, flags=flags)
        assert np.array_equal(aa, ab), flags
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32)), flags


@pytest.mark.parametrize("cli", ["c2torus.cli", "old_t07a.cli", "rect_test.cli", "p4_t06Alt.cli", "c4InSphere.cli"])
def test_ignored_command_scenes_parity(cli):
    """Scenes with commands readRTFile does not know (`torus`, `backgroun`, `color` / `rect`,
    `marble2`: reported and skipped, myRTFileReader.java:343-345) and c4InSphere (moonmap4k.jpg,
    11 point lights: lights past the wave-level cull's 8) render as the oracle does."""
    g, o, (rg, ag), (ro, ao) = both(cli, 96, 96, 1)
    assert_exact_decisions(compare(rg, ag, ro, ao))


def _many_entries_scene(n_side):
    """n_side^2 spheres (alternately diffuse and mirror) over a ground quad, point + spot lights:
    more than 64 objList entries when n_side >= 9."""
    lines = ["fov 60", "background 0.1 0.1 0.2", "point_light 3 6 2 .6 .6 .6",
             "spotlight -3 7 -4  0.3 -1 -0.2  20 45  .5 .5 .5", "diffuse .6 .6 .6 .1 .1 .1",
             "begin quad", "vertex -30 -1 -60", "vertex 30 -1 -60", "vertex 30 -1 10", "vertex -30 -1 10", "end"]
    for i in range(n_side):
        for j in range(n_side):
            if (i + j) % 2:
                lines.append(f"shiny .2 .2 .6 .05 .05 .1 .5 .5 .5 20 0.4")
            else:
                lines.append(f"diffuse .8 .{i % 9 + 1} .{j % 9 + 1} .1 .1 .1")
            lines.append(f"sphere 0.35 {-3.2 + 0.8 * j:.2f} {-0.6 + 0.1 * i:.2f} {-4.5 - 0.9 * i:.2f}")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("n_side", [8, 9])
def test_more_than_64_top_level_entries(tmp_path, n_side):
    """objList with 65 (8x8 spheres + a quad) and 82 entries: past the wave-level shadow cull's
    64-entry candidate word every entry is scanned (no shift past 63, no endless loop). The
    default render equals the per-lane scan, the reference's full scan and the oracle."""
    (tmp_path / "many.cli").write_text(_many_entries_scene(n_side))
    g = rt.Scene.load_cli("many.cli", scene_dir=tmp_path, textures={})
    assert g.info()["objects"] == n_side * n_side + 1
    ra, aa = g.render(64, 64, spp=2, seed=SEED)
    for flags in (rt.RENDER_NOWAVECULL, rt.RENDER_NOCULL, rt.RENDER_GENERIC):
        rb, ab = g.render(64, 64, spp=2, seed=SEED, flags=flags)
        assert np.array_equal(aa, ab), flags
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32)), flags
    o = OracleScene(tmp_path, "many.cli")
    ro, ao, _ = o.render(64, 64, spp=2, seed=SEED)
    assert_exact_decisions(compare(ra, aa, ro, ao))


@pytest.mark.parametrize("cli,W,spp", [("plnts3ColsBunnies.cli", 96, 4), ("c2clear.cli", 96, 1), ("trTrans.cli", 96, 2),
                                       ("c3_bun69k.cli", 128, 4), ("p2_t07.cli", 96, 2), ("old_t10.cli", 96, 4),
                                       ("t11.cli", 64, 2), ("p3_t11_sierp.cli", 64, 1), ("c4InSphere.cli", 96, 1),
                                       ("t01.cli", 96, 1)])
def test_wavefront_renders_identically(cli, W, spp):
    """RT_RENDER_WAVEFRONT (level-synchronous shading: one launch per generation of the shading tree,
    children compacted into the next level's queue, frames folded bottom up) renders the monolithic
    kernel's image bit for bit: glass (Fresnel and simple), mirrors, DOF, fisheye, photon map,
    instances, 1 spp -- in the scene's variant and the generic one."""
    scenes.ensure_bun69k()
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    ra, aa = g.render(W, W, spp=spp, seed=SEED)
    for flags in (rt.RENDER_WAVEFRONT, rt.RENDER_WAVEFRONT | rt.RENDER_GENERIC):
        rb, ab = g.render(W, W, spp=spp, seed=SEED, flags=flags)
        assert np.array_equal(aa, ab), flags
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32)), flags


def test_wavefront_undersized_queue_is_an_error(monkeypatch):
    """The level-synchronous path's device guards are loud: with the queue
    capacity deliberately undersized (DISTRAYTRACER_WF_QCAP_DIV) the device drops children past it,
    sets its error word and the render returns RT_E_HIP instead of a wrong image; at the true
    capacity the same scene renders the plain image."""
    g = rt.Scene.load_cli("plnts3ColsBunnies.cli", textures=scenes.prepare("plnts3ColsBunnies.cli"))
    ra, aa = g.render(96, 96, spp=2, seed=SEED)
    monkeypatch.setenv("DISTRAYTRACER_WF_QCAP_DIV", "8")
    with pytest.raises(rt.RTError, match="dropped"):
        g.render(96, 96, spp=2, seed=SEED, flags=rt.RENDER_WAVEFRONT)
    monkeypatch.setenv("DISTRAYTRACER_WF_QCAP_DIV", "1")
    rb, ab = g.render(96, 96, spp=2, seed=SEED, flags=rt.RENDER_WAVEFRONT)
    assert np.array_equal(aa, ab) and np.array_equal(ra.view(np.uint32), rb.view(np.uint32))


def test_pixel_waves_render_identically():
    """RT_RENDER_PIXEL_WAVES (one pixel per wave, 64 sample lanes, those past spp idle; the multi-GPU
    split's per-pixel mode) renders the plain image -- spp a power of two and not -- and is refused at
    spp = 1, where the 64-lane layout would sum a pixel's single colour from 0."""
    g = rt.Scene.load_cli("plnts3ColsBunnies.cli", textures=scenes.prepare("plnts3ColsBunnies.cli"))
    for spp in (2, 6):
        ra, aa = g.render(64, 64, spp=spp, seed=SEED)
        rb, ab = g.render(64, 64, spp=spp, seed=SEED, flags=rt.RENDER_PIXEL_WAVES)
        assert np.array_equal(aa, ab), spp
        assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32)), spp
    with pytest.raises(rt.RTError, match="spp >= 2"):
        g.render(64, 64, spp=1, seed=SEED, flags=rt.RENDER_PIXEL_WAVES)


def test_wavefront_c4_oracle_parity():
    """The level-synchronous path against the oracle on C4's scene (glass bunnies, mirrors, textures)."""
    g, o, _, (ro, ao) = both("plnts3ColsBunnies.cli", 160, 160, 2, seed=0x5EED0004)
    rg, ag = g.render(160, 160, spp=2, seed=0x5EED0004, flags=rt.RENDER_WAVEFRONT)
    assert_exact_decisions(compare(rg, ag, ro, ao))


@pytest.mark.parametrize("cli,W,spp", [("c3_bun69k.cli", 128, 4), ("plnts3ColsBunnies.cli", 96, 4), ("t11.cli", 64, 2),
                                       ("p2_t07.cli", 96, 2), ("old_t10.cli", 96, 4), ("t01.cli", 96, 1),
                                       ("p3_t11_sierp.cli", 64, 1)])
def test_sample_waves_render_identically(cli, W, spp):
    """rt_render_pixels_device (one sample per wave, each pixel summed in sample order afterwards: the
    multi-GPU split's heaviest tiles) writes exactly the listed pixels of the plain render, and no
    other: glass, photon map, DOF, fisheye (untraced samples outside the image circle), 1 spp, instances."""
    import torch

    scenes.ensure_bun69k()
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    ra, aa = g.render(W, W, spp=spp, seed=SEED)
    rng = np.random.default_rng(W + spp)
    pix = np.unique(rng.integers(0, W * W, size=W * W // 5)).astype(np.int32)
    rgb = torch.full((W * W, 3), -1.0, device="cuda")
    argb = torch.zeros(W * W, dtype=torch.int32, device="cuda")
    g.render_pixels_device(rt.params(W, W, spp=spp, seed=SEED), pix, rgb.data_ptr(), argb.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rb, ab = rgb.cpu().numpy(), argb.cpu().numpy()
    mask = np.zeros(W * W, bool)
    mask[pix] = True
    assert np.array_equal(ab[mask], aa.reshape(-1)[mask])
    assert np.array_equal(rb[mask].view(np.uint32), ra.reshape(-1, 3)[mask].view(np.uint32))
    assert (rb[~mask] == -1.0).all()


def test_photon_shards_merge_to_the_full_prepass(tmp_path):
    """Multi-GPU photon pre-pass (8(e)): shards shot separately and merged in rank order give
    the single-GPU photon_list bit for bit, and the same image."""
    from distraytracer_old_amd import multigpu
    src = (scenes.SCENE_DIR / "t11.cli").read_text().replace("diffuse_photons  1000000  200 0.1",
                                                             "diffuse_photons  30001  50 0.1")
    (tmp_path / "t11s.cli").write_text(src)
    seed = 0x5EED0005
    full = rt.Scene.load_cli("t11s.cli", scene_dir=tmp_path, textures={})
    full.build_photons(seed)
    fp, fw = full.photons()
    sh = rt.Scene.load_cli("t11s.cli", scene_dir=tmp_path, textures={})
    shards = []
    for r in range(3):
        first, n = multigpu.photon_shard(r, 3, 30001)
        shards.append(sh.shoot_photons(seed, first, n))
    mp, mw = multigpu.merge_photon_shards(shards)
    assert np.array_equal(mp, fp) and np.array_equal(mw, fw)
    sh.set_photons(mp, mw)
    a = full.render(64, 64, spp=2, seed=seed)
    b = sh.render(64, 64, spp=2, seed=seed)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0])


def test_rank_bands_equal_full_image_rows():
    """A rank's banded tile (multi-GPU partition, 8(e)) is exactly its rows of the 1-GPU image."""
    from distraytracer_old_amd import multigpu
    tex = scenes.prepare("c3_bun69k.cli")
    g = rt.Scene.load_cli("c3_bun69k.cli", textures=tex)
    full, af = g.render(256, 256, spp=4, seed=SEED)
    for world, rank in [(8, 3), (3, 2)]:
        r0, r1, step, band = multigpu.rows_of(rank, world, 256)
        tile, at = g.render(256, 256, spp=4, seed=SEED, rows=(r0, r1), row_step=step, row_band=band)
        rows = multigpu.image_rows(rank, world, 256)
        assert np.array_equal(tile, full[rows]) and np.array_equal(at, af[rows])


def test_tile_schedule_does_not_change_the_image():
    """The longest-first tile dispatch orders -- the probe's (1st render of a layout, which
    also measures its waves) and the measured one (2nd render on) -- render bit-identically
    to row-major."""
    g = rt.Scene.load_cli("c3_bun69k.cli", textures=scenes.prepare("c3_bun69k.cli"))
    b, ab = g.render(512, 512, spp=2, seed=SEED, flags=rt.RENDER_ROWMAJOR)
    for _ in range(3):  # probe order + measuring, then measured order twice
        a, aa = g.render(512, 512, spp=2, seed=SEED)
        assert np.array_equal(aa, ab) and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _maps_equal(a, b):
    assert rt.photon_maps_equal(a, b)


def test_gpu_photon_map_build_equals_host_build(tmp_path, monkeypatch):
    """The photon map's search structure built on the GPU (photon_build.hip, the default) is the
    host build's (photon.cpp) node for node, and renders the same image bit for bit."""
    src = (scenes.SCENE_DIR / "t11.cli").read_text().replace("diffuse_photons  1000000  200 0.1",
                                                             "diffuse_photons  60000  50 0.1")
    (tmp_path / "t11m.cli").write_text(src)
    seed = 0x5EED0005
    g = rt.Scene.load_cli("t11m.cli", scene_dir=tmp_path, textures={})
    g.build_photons(seed)
    monkeypatch.setenv("DISTRAYTRACER_PHOTON_BUILD", "host")
    h = rt.Scene.load_cli("t11m.cli", scene_dir=tmp_path, textures={})
    h.build_photons(seed)
    monkeypatch.delenv("DISTRAYTRACER_PHOTON_BUILD")
    assert g.info()["photons"] > 1000
    _maps_equal(g.photon_map(), h.photon_map())
    a = g.render(64, 64, spp=2, seed=seed)
    b = h.render(64, 64, spp=2, seed=seed)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))


@pytest.mark.parametrize("n", [25, 49, 1000, 262147])
def test_gpu_photon_map_build_ties_and_sizes(tmp_path, monkeypatch, n):
    """Adversarial photon lists through rt_photons_set: heavy coordinate ties (a coarse grid),
    signed zeros, a range straddling one leaf -- GPU build == host build."""
    (tmp_path / "t11m.cli").write_text((scenes.SCENE_DIR / "t11.cli").read_text())
    rng = np.random.default_rng(n)
    pos = rng.integers(-3, 4, size=(n, 3)).astype(np.float64) * 0.25
    pos[rng.random((n, 3)) < 0.2] = -0.0
    pwr = rng.random((n, 3))
    maps = []
    for mode in ("gpu", "host"):
        if mode == "host":
            monkeypatch.setenv("DISTRAYTRACER_PHOTON_BUILD", "host")
        s = rt.Scene.load_cli("t11m.cli", scene_dir=tmp_path, textures={})
        s.set_photons(pos, pwr)
        maps.append(s.photon_map())
        s.close()
    monkeypatch.delenv("DISTRAYTRACER_PHOTON_BUILD")
    _maps_equal(maps[0], maps[1])


@pytest.mark.parametrize("cli,W,spp", [("plnts3ColsBunnies.cli", 128, 4), ("p2_t05.cli", 96, 2), ("c2clear.cli", 96, 1),
                                       ("p2_t07.cli", 96, 2), ("c3shinyBall.cli", 96, 1)])
def test_top_level_culling_does_not_change_the_image(cli, W, spp):
    """Bounding-sphere culling of top-level spheres / cylinders / boxes (closest and any-hit)
    renders bit-identically to testing every top-level primitive (RT_RENDER_NOCULL)."""
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    a, aa = g.render(W, W, spp=spp, seed=SEED)
    b, ab = g.render(W, W, spp=spp, seed=SEED, flags=rt.RENDER_NOCULL)
    assert np.array_equal(aa, ab) and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("cli,W,spp", [("plnts3ColsBunnies.cli", 96, 2), ("c5Fish.cli", 80, 1),
                                       ("planets3Ortho.cli", 80, 1), ("t11.cli", 64, 1)])
def test_refine_passes(cli, W, spp):
    """`refine on` (myScene.setRefine + draw, myScene.java:796-803,1481-1531): the reference's
    steps for the image size; after each pass every pixel holds the colour of the pass's sample
    at the top-left of its step x step span (writePxlSpan; (0,0) skipped after the first pass),
    and the last pass leaves exactly the plain render's image."""
    g = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    assert g.refine_steps(300, 300) == [16, 8, 4, 2, 1]
    assert g.refine_steps(1024, 1024) == [64, 32, 16, 8, 4, 2, 1]
    full, fa = g.render(W, W, spp=spp, seed=SEED)
    rgb = np.zeros((W, W, 3), np.float32)
    argb = np.zeros((W, W), np.int32)
    steps = g.refine_steps(W, W)
    assert steps[-1] == 1 and len(steps) >= 2
    for k, s in enumerate(steps):
        g.render_pass(W, W, s, k > 0, rgb, argb, spp=spp, seed=SEED)
        idx = (np.arange(W) // s) * s
        assert np.array_equal(argb, fa[np.ix_(idx, idx)]), (cli, s)
        assert np.array_equal(rgb.view(np.uint32), full[np.ix_(idx, idx)].view(np.uint32)), (cli, s)


def test_refine_off_is_one_pass():
    g = rt.Scene.load_cli("c3_bun69k.cli", textures=scenes.prepare("c3_bun69k.cli"))
    assert g.refine_steps(1024, 1024) == [1]
