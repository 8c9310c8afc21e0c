"""bench.py's N-GPU step path on the HIP kernel (VERDICT r01 Next #2): tools/rank_check.py
runs multigpu.RankRenderer + FrameExchange (+ the sharded photon pre-pass) as 2 ranks over
gloo sharing device 0 (tiles staged to host), and as 1 rank; the assembled 2-rank frame (float
RGB and ARGB) must equal the 1-rank image bit for bit, and bench.py --gpus 2 must print a 2-rank
line.

These tests start child processes, so conftest.py runs them before any test of the session
touches the GPU in the pytest process (no exec from a GPU-initialised process)."""
import json
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
pytestmark = [pytest.mark.gpu, pytest.mark.spawns]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, nproc, tmp, name):
    out = tmp / f"{name}.npz"
    tool = [str(REPO / "tools" / "rank_check.py"), *args, "--out", str(out)]
    if nproc == 1:
        cmd = [sys.executable, *tool]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", *tool]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = np.load(out)
    return d["rgb"], d["argb"]


@pytest.mark.parametrize("partition", ["tiles", "bands"])
@pytest.mark.parametrize("args", [
    ["--cli", "c3_bun69k.cli", "--size", "256", "--spp", "4"],
    ["--cli", "t11.cli", "--size", "96", "--spp", "2", "--seed", str(0x5EED0005)],  # sharded photon pre-pass
], ids=["c3", "t11_photons"])
def test_two_rank_step_equals_one_rank_image(tmp_path, args, partition):
    """Cost-balanced tiles (the default: rank 0's measured costs broadcast, rt_render_tiles_device,
    pixels packed / scattered) and interleaved bands."""
    one, one_argb = _run(args, 1, tmp_path, "one")
    two, two_argb = _run(args + ["--partition", partition], 2, tmp_path, "two")
    assert one.shape == two.shape
    assert np.array_equal(one.view(np.uint32), two.view(np.uint32))
    # the reference's output, rndrdImg.pixels (myObjShader.java:671): rank 0's assembled ARGB
    # frame equals the 1-GPU frame's ints
    assert one_argb.shape == one.shape[:2] and np.array_equal(one_argb, two_argb)


def test_bench_gpus2_prints_a_two_rank_line():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and "rehearsal" in d
