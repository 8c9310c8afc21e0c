"""Generate the golden fixtures in tests/golden/ with the oracle (CPU restatement).

The Java reference cannot run here (no JDK), so these vectors are oracle outputs
pinned by the hand-derived KATs (tests/test_oracle.py); they freeze the oracle's
behaviour so the GPU path can be checked without running the oracle, and any
oracle change is caught. Each fixture: a crop of a config render at a fixed
seed: rgb float32 [h,w,3] (clamped myColor values) + argb int32 [h,w].

usage: python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from distraytracer_old_amd import scenes  # noqa: E402
from oracle.oracle import OracleScene  # noqa: E402

# name: (cli, W, H, spp, seed, row0, row1, col0, col1)
FIXTURES = {
    "c1_t01_256": ("t01.cli", 256, 256, 1, 0x5EED0001, 96, 160, 96, 160),
    "c2_shiny_512": ("c3shinyBall.cli", 512, 512, 1, 0x5EED0001, 200, 264, 224, 288),
    "c3_bun69k_256": ("c3_bun69k.cli", 256, 256, 4, 0x5EED0001, 96, 160, 96, 160),
    "c4_planets_192": ("plnts3ColsBunnies.cli", 192, 192, 2, 0x5EED0004, 80, 144, 40, 104),
    "f_disk_p2t05": ("p2_t05.cli", 96, 96, 4, 0x5EED0001, 0, 96, 0, 96),
    "f_dof_p2t07": ("p2_t07.cli", 96, 96, 4, 0x5EED0001, 0, 96, 0, 96),
    "f_refr_c2clear": ("c2clear.cli", 96, 96, 1, 0x5EED0001, 0, 96, 0, 96),
    "f_motion_p2t03": ("p2_t03.cli", 96, 96, 4, 0x5EED0001, 0, 96, 0, 96),
}


def render(name):
    cli, W, H, spp, seed, r0, r1, c0, c1 = FIXTURES[name]
    o = OracleScene(scenes.SCENE_DIR, cli, scenes.prepare(cli))
    rgb, argb, _ = o.render(W, H, spp=spp, seed=seed, rows=(r0, r1))
    return rgb[:, c0:c1].copy(), argb[:, c0:c1].copy()


if __name__ == "__main__":
    for name in FIXTURES:
        rgb, argb = render(name)
        np.savez_compressed(HERE / f"{name}.npz", rgb=rgb, argb=argb, spec=np.array(FIXTURES[name][1:], dtype=np.int64),
                            cli=np.array(FIXTURES[name][0]))
        print(name, rgb.shape, float(rgb.mean()))
