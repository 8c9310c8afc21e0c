"""Statistical pin against the reference's own output: the reference's
300x300 render of data/t11.cli (t11c.png; stochastic: Java RNG, 1 M photons per light)
reduced to 10x10-pixel block means (tests/golden/t11c_refstats.npz, made by
make_refstats.py). The oracle and the GPU render the same scene with their own keyed
RNG; the images must agree statistically: channel means within 2 %, block RMS < 0.02,
block correlation > 0.995 (oracle at 50 spp measured: 0.5 %, 0.0107, 0.9992).
"""
from pathlib import Path

import numpy as np
import pytest

from distraytracer_old_amd import scenes

GOLD = Path(__file__).resolve().parent / "golden" / "t11c_refstats.npz"


def blocks(rgb, b=10):
    h, w, c = rgb.shape
    return rgb.reshape(h // b, b, w // b, b, c).mean((1, 3))


def check(rgb):
    ref = np.load(GOLD)
    rb = blocks(np.asarray(rgb, dtype=np.float64).clip(0, 1))
    mean = rb.mean((0, 1))
    rel = np.abs(mean - ref["mean"]) / ref["mean"]
    rms = float(np.sqrt(((rb - ref["blocks"]) ** 2).mean()))
    corr = float(np.corrcoef(rb.ravel(), ref["blocks"].ravel())[0, 1])
    assert rel.max() < 0.02, (mean, ref["mean"])
    assert rms < 0.02, rms
    assert corr > 0.995, corr
    return rel, rms, corr


def test_oracle_t11_matches_reference_render():
    from oracle.oracle import OracleScene
    o = OracleScene(scenes.SCENE_DIR, "t11.cli", scenes.prepare("t11.cli"))
    o.build_photons(0x5EED0005)
    rgb, _, _ = o.render(300, 300, spp=10, seed=0x5EED0005, threads=8)
    print(check(rgb))


@pytest.mark.gpu
def test_gpu_t11_matches_reference_render():
    from distraytracer_old_amd import rt
    g = rt.Scene.load_cli("t11.cli", textures=scenes.prepare("t11.cli"))
    rgb, _ = g.render(300, 300, spp=0, seed=0x5EED0005)  # the scene's rays_per_pixel (50)
    print(check(rgb))
