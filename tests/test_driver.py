"""Headless driver tools/rtrender (SURVEY 8(b) caller 1): .cli -> C ABI -> PNG."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def build():
    subprocess.run(["bash", str(REPO / "tools" / "build_rtrender.sh")], check=True, capture_output=True)
    return REPO / "tools" / "rtrender"


def test_driver_builds_and_fails_loudly_without_gpu():
    exe = build()
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_driver_t01_png_kat(tmp_path):
    from PIL import Image
    exe = build()
    out = tmp_path / "t01.png"
    r = subprocess.run([str(exe), str(REPO / "scenes"), "t01.cli", "-o", str(out), "-rgb", str(tmp_path / "t01.f32")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    img = np.asarray(Image.open(out).convert("RGB"))
    assert img.shape == (300, 300, 3)
    assert tuple(img[150, 150]) == (0x9E, 0, 0)  # t01 KAT: 0xFF9E0000
    rgb = np.fromfile(tmp_path / "t01.f32", dtype=np.float32).reshape(300, 300, 3)
    assert abs(rgb[150, 150, 0] - 0.621637) < 1e-6


@pytest.mark.gpu
def test_driver_textured_scene_matches_python_path(tmp_path):
    from PIL import Image
    from distraytracer_old_amd import rt, scenes
    exe = build()
    targs = subprocess.run(["python3", str(REPO / "tools" / "textures_to_ppm.py"), "plnts3ColsBunnies.cli",
                            str(tmp_path / "tex")], capture_output=True, text=True, check=True).stdout.split()
    out = tmp_path / "p.png"
    scenes.ensure_bun69k()
    r = subprocess.run([str(exe), str(REPO / "scenes"), "plnts3ColsBunnies.cli", "-w", "96", "-h", "96", "-spp", "1",
                        "-seed", str(0x5EED0004), "-o", str(out), *targs], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    img = np.asarray(Image.open(out).convert("RGB")).astype(np.int64)
    g = rt.Scene.load_cli("plnts3ColsBunnies.cli", textures=scenes.prepare("plnts3ColsBunnies.cli"))
    _, argb = g.render(96, 96, spp=1, seed=0x5EED0004)
    a = argb.view(np.uint32)
    ref = np.stack([(a >> 16) & 255, (a >> 8) & 255, a & 255], -1).astype(np.int64)
    assert np.array_equal(img, ref)
