"""Scene inputs: the synthetic bun69k stand-in and texture decoding."""
import hashlib

import numpy as np

from distraytracer_old_amd import scenes


def test_bun69k_shape_and_bbox():
    t = scenes.synth_bun69k()
    assert t.shape == (69451, 3, 3)
    base = scenes._parse_tris(scenes.SCENE_DIR / "bun500.cli")
    assert base.shape == (966, 3, 3)
    np.testing.assert_allclose(t.reshape(-1, 3).min(0), base.reshape(-1, 3).min(0))
    np.testing.assert_allclose(t.reshape(-1, 3).max(0), base.reshape(-1, 3).max(0))


def test_bun69k_file_is_deterministic():
    p = scenes.ensure_bun69k()
    h1 = hashlib.sha256(p.read_bytes()).hexdigest()
    t = scenes.synth_bun69k()
    assert np.array_equal(t, scenes.synth_bun69k())
    lines = p.read_text().splitlines()
    assert sum(1 for l in lines if l == "begin") == 69451
    assert h1 == hashlib.sha256(p.read_bytes()).hexdigest()


def test_texture_names_and_decode():
    names = scenes.texture_names("plnts3ColsBunnies.cli")
    assert names[0] == "nightSky.png" and "earthMap.jpg" in names and len(names) == 6
    a = scenes.load_texture("checkersphere.jpg")
    assert a.dtype == np.uint8 and a.shape == (512, 512, 3)
