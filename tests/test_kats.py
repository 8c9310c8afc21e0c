"""Reference-independent known answers (tests/golden/kats.json, derived by tests/golden/make_kats.py
in plain float64 Python from the Java formulas, without the oracle or the product): the glass
shaders (calcSimpleTransClr, calcTransClr with a real Fresnel split), the spot fall-off band and
disk-light sampling, at 300 x 300, 1 spp. The oracle (CPU) and the HIP path (-m gpu) must reproduce
each pixel: float32 RGB within 2e-6 of the derived double colour (host libm vs fdlibm trig: an ulp),
and the ARGB int exactly (the script keeps every channel 1e-9 away from a truncation step)."""
import importlib.util
import json
from pathlib import Path

import numpy as np
import pytest

from distraytracer_old_amd import scenes

GOLDEN = Path(__file__).resolve().parent / "golden"
KATS = json.loads((GOLDEN / "kats.json").read_text())
TOL = 2e-6


def _make_kats():
    spec = importlib.util.spec_from_file_location("make_kats", GOLDEN / "make_kats.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _scene(kat, tmp_path):
    """(scene_dir, cli, textures) of a KAT's scene; trTrans_plain.cli is written to tmp_path."""
    if kat["cli"] == "trTrans_plain.cli":
        (tmp_path / kat["cli"]).write_text(_make_kats().scene_text(kat["cli"]))
        return tmp_path, kat["cli"], {}
    return scenes.SCENE_DIR, kat["cli"], scenes.prepare(kat["cli"])


def _check(kat, rgb, argb):
    got = rgb[0, kat["col"]].astype(np.float64)
    assert np.abs(got - np.asarray(kat["rgb"])).max() <= TOL, (kat["name"], got, kat["rgb"])
    assert int(argb[0, kat["col"]]) == kat["argb"], (kat["name"], hex(int(argb[0, kat["col"]]) & 0xFFFFFFFF))


def test_kat_fixture_is_the_derivation():
    """kats.json is what make_kats.py derives (the script is the fixture's source of truth)."""
    m = _make_kats()
    for kat in KATS["kats"]:
        sc = m.load(m.scene_text(kat["cli"]), KATS["W"], KATS["H"])
        assert sc.pixel(kat["row"], kat["col"], KATS["seed"]) == kat["rgb"], kat["name"]


@pytest.mark.parametrize("kat", KATS["kats"], ids=[k["name"] for k in KATS["kats"]])
def test_oracle_reproduces_kat(kat, tmp_path):
    from oracle.oracle import OracleScene

    d, cli, tex = _scene(kat, tmp_path)
    o = OracleScene(d, cli, tex)
    rgb, argb, _ = o.render(KATS["W"], KATS["H"], spp=1, seed=KATS["seed"], rows=(kat["row"], kat["row"] + 1))
    _check(kat, rgb, argb)


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS["kats"], ids=[k["name"] for k in KATS["kats"]])
def test_gpu_reproduces_kat(kat, tmp_path):
    from distraytracer_old_amd import rt

    d, cli, tex = _scene(kat, tmp_path)
    with rt.Scene.load_cli(cli, scene_dir=d, textures=tex) as g:
        rgb, argb = g.render(KATS["W"], KATS["H"], spp=1, seed=KATS["seed"], rows=(kat["row"], kat["row"] + 1))
    _check(kat, rgb, argb)
