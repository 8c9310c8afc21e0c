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


@pytest.mark.parametrize("name,png", [("t01.png", "t01.png"), ("t01", "t01.png"), ("a.b.png", "a.b.png"),
                                      ("dir.x/t01", "dir.png"), ("abc.", "abc..png"), ("x.y.", "x.y..png"),
                                      ("scenes/t03.cli", "scenes/t03.png"), (".png", ".png")])
def test_png_name_rule(name, png):
    """myScene.saveFile: split("\\.(?=[^\\.]+$)")[0] + ".png" (myScene.java:1188-1192)."""
    from distraytracer_old_amd import rt
    assert rt.png_name(name) == png


@pytest.mark.gpu
def test_driver_default_output_name(tmp_path):
    """no -o: pics.<date>/<write name>.png (t01.cli ends with `write t01.png`); -nodir: cwd."""
    exe = build()
    r = subprocess.run([str(exe), str(REPO / "scenes"), "t01.cli", "-w", "32", "-h", "32"], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    pics = [p for p in tmp_path.iterdir() if p.name.startswith("pics.")]
    assert len(pics) == 1 and (pics[0] / "t01.png").exists(), list(tmp_path.iterdir())
    r = subprocess.run([str(exe), str(REPO / "scenes"), "t01.cli", "-w", "32", "-h", "32", "-nodir"], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0 and (tmp_path / "t01.png").exists(), r.stderr


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
