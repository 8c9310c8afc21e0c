"""Quick GPU timing probe: kernel time (HIP events) for the BASELINE configs."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distraytracer_old_amd import rt, scenes  # noqa: E402

cfgs = sys.argv[1:] or ["C2", "C3"]
for c in cfgs:
    cli, W, H, spp, seed = scenes.CONFIGS[c]
    t0 = time.time()
    s = rt.Scene.load_cli(cli)
    t1 = time.time()
    _, _, st = s.render_count(W, H, spp=spp, seed=seed)
    rays = st["camera"] + st["shadow"] + st["refl"] + st["refr"]
    ms = s.time_render(W, H, spp=spp, seed=seed, warmup=1, iters=2)
    print(f"{c} {cli} {W}x{H}x{spp}: load {t1-t0:.2f}s kernel {ms:.1f} ms rays {rays} -> {rays/ms/1e3:.1f} Mray/s {st}",
          flush=True)
