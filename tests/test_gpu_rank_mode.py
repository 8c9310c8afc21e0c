"""The native one-process-per-GPU group at world > 1 (rt_group_create_comm; VERDICT r05 Next #1):
tools/group_rank_check.py runs 2 and 3 real ranks over the host transport (rt_comm_create_host on
gloo; every rank on device 0), so the rank-mode code that bench.py --gpus N and the JNI N-GPU draw()
(myScene.java:1481-1531) use executes before any multi-GPU run: the argument check, rank 0's cost
broadcast, the plan check after every cut (each sender's slab offset / count / pixel-list hash against
rank 0's receive side), the rebalance all-gather, the exchange into rank 0's slab and the scatter.
Every frame -- blocking into host buffers and pipelined into device buffers -- equals rt_render bit
for bit; the sharded photon pre-pass (rt_photons_build_comm) equals rt_photons_build bit for bit;
ranks given different frames all fail instead of hanging. On a machine with >= 2 GPUs the same
check runs over RCCL (one device per rank).

These tests start child processes, so conftest.py runs them before this process touches the GPU."""
import json
import socket
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
pytestmark = [pytest.mark.gpu, pytest.mark.spawns]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, args, tmp):
    out = tmp / "report.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(REPO / "tools" / "group_rank_check.py"),
           *args, "--out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    return json.loads(out.read_text())


def _assert_checks(rep):
    bad = [c for c in rep["checks"] if not c[1]]
    assert not bad, bad


CASES = {
    "c3": ["--cli", "c3_bun69k.cli", "--width", "320", "--height", "256", "--spp", "4"],
    "t11": ["--cli", "t11.cli", "--width", "256", "--height", "256", "--spp", "4", "--seed", str(0x5EED0005)],
}


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", list(CASES))
def test_rank_mode_host_transport_reassembles_the_frame(tmp_path, case, world):
    rep = _run(world, CASES[case] + ["--transport", "host"], tmp_path)
    _assert_checks(rep)
    assert rep["comm"]["transport"] == "host" and rep["world"] == world
    assert rep["group_info"]["plan_checks"] == 1  # at creation; "plan checked after every cut" covers the re-cuts
    assert "plan checked after every cut" in [c[0] for c in rep["checks"]]
    assert rep["split_tiles"] > 0  # heavy 0.1 / 64 slots: the one-sample-per-wave path runs too
    names = [c[0] for c in rep["checks"]]
    assert "every frame == rt_render bit for bit" in names
    if case == "t11":
        assert "photon_list and map == rt_photons_build" in names


def test_rank_mode_host_transport_c4_scene(tmp_path):
    """C4's variant (glass, image / marble textures, spot lights) in rank mode: 2 ranks."""
    rep = _run(2, ["--cli", "plnts3ColsBunnies.cli", "--width", "256", "--height", "256", "--spp", "2",
                   "--seed", str(0x5EED0004), "--transport", "host"], tmp_path)
    _assert_checks(rep)
    assert "every frame == rt_render bit for bit" in [c[0] for c in rep["checks"]]


def test_rank_mode_mismatched_frame_fails_on_every_rank(tmp_path):
    rep = _run(2, CASES["c3"] + ["--transport", "host", "--mismatch"], tmp_path)
    _assert_checks(rep)
    assert "different frame" in rep["create_error"]


def test_rank_mode_rccl_two_gpus(tmp_path):
    """RCCL rank mode, one device per rank: only where two GPUs are visible (the one-GPU box
    cannot run two RCCL ranks)."""
    sys.path.insert(0, str(REPO))
    import bench

    if bench.visible_gpus() < 2:
        pytest.skip("needs 2 GPUs")
    rep = _run(2, CASES["c3"] + ["--transport", "rccl"], tmp_path)
    _assert_checks(rep)
    assert rep["comm"]["transport"] == "rccl"
