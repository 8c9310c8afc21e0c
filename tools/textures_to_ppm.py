#!/usr/bin/env python3
"""Decode the textures a .cli references (same Pillow decode as the tests, scenes.prepare) into
binary PPM files for tools/rtrender; prints the matching -tex arguments.

  python tools/textures_to_ppm.py plnts3ColsBunnies.cli /tmp/tex
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distraytracer_old_amd import scenes  # noqa: E402

cli, out = sys.argv[1], Path(sys.argv[2])
out.mkdir(parents=True, exist_ok=True)
args = []
for name, rgb in scenes.prepare(cli).items():
    p = out / (Path(name).name + ".ppm")
    with open(p, "wb") as f:
        f.write(b"P6 %d %d 255\n" % (rgb.shape[1], rgb.shape[0]))
        f.write(rgb.tobytes())
    args += ["-tex", f"{name}={p}"]
print(" ".join(args))
