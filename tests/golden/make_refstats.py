#!/usr/bin/env python3
"""Statistical fixture from the reference's own render ("t11c.png ... usable only
as a statistical sanity check at 300x300").

/root/reference/t11c.png is the reference's 300x300 output of data/t11.cli (Cornell box:
photon map, disk light, mirror + glass spheres; stochastic, Java RNG). This script stores
only derived statistics -- 10x10-pixel block means (30x30x3) and channel means -- in
t11c_refstats.npz. Run here (the reference is not on the GPU box):

    python tests/golden/make_refstats.py
"""
from pathlib import Path

import numpy as np
from PIL import Image

HERE = Path(__file__).resolve().parent


def blocks(rgb, b=10):
    h, w, c = rgb.shape
    return rgb.reshape(h // b, b, w // b, b, c).mean((1, 3))


def main():
    ref = np.asarray(Image.open("/root/reference/t11c.png").convert("RGB")).astype(np.float64) / 255.0
    np.savez_compressed(HERE / "t11c_refstats.npz", blocks=blocks(ref), mean=ref.mean((0, 1)),
                        source=np.array("reference t11c.png (300x300 render of data/t11.cli), 10x10 block means"))
    print("mean", ref.mean((0, 1)))


if __name__ == "__main__":
    main()
