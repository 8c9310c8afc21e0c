"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py):
the oracle must reproduce them (CPU), and the HIP path must match them within
the stated tolerance (GPU) -- the GPU check needs no oracle at run time."""
import numpy as np
import pytest

from distraytracer_old_amd import scenes
from tests.golden.make_golden import FIXTURES, render
from tests.parity import TOL, assert_exact_decisions, compare

import pathlib

GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def load(name):
    z = np.load(GOLD / f"{name}.npz", allow_pickle=False)
    return z["rgb"], z["argb"]


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_oracle_reproduces_golden(name):
    rgb, argb = render(name)
    g_rgb, g_argb = load(name)
    np.testing.assert_allclose(rgb, g_rgb, atol=1e-6)
    assert np.array_equal(argb, g_argb)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_gpu_matches_golden(name):
    from distraytracer_old_amd import rt

    cli, W, H, spp, seed, r0, r1, c0, c1 = FIXTURES[name]
    s = rt.Scene.load_cli(cli, textures=scenes.prepare(cli))
    rgb, argb = s.render(W, H, spp=spp, seed=seed, rows=(r0, r1))
    g_rgb, g_argb = load(name)
    c = compare(rgb[:, c0:c1], argb[:, c0:c1], g_rgb, g_argb, tol=TOL)
    assert_exact_decisions(c)
