"""The host transport of rt_comm (include/distraytracer.h ABI 7) on CPU: world 1, 2 and 3 processes
over gloo, each calling the library's collectives (rt_comm_selftest: all-gather, a broadcast from
every rank, the group's ranks-to-rank-0 exchange pattern) through the ctypes callbacks. This is the
transport the one-process-per-GPU group runs over in tests/test_gpu_rank_mode.py; here its bindings
are checked without a GPU. A rank whose callback fails makes its call fail (no hang)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distraytracer_old_amd import rt


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode):
    import sys
    from datetime import timedelta
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from distraytracer_old_amd import rt

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=timedelta(seconds=60 if mode == "ok" else 8))
    try:
        with rt.Comm.host(dist) as c:
            info = c.info()
            assert info == {"rank": rank, "world": world, "transport": "host", "device": -1}, info
            if mode == "ok":
                for n in (1, 1031, 70001):
                    c.selftest(n)
                q.put((rank, "ok"))
            else:  # a broken callback on the last rank: its call raises instead of hanging
                if rank == world - 1:
                    cbs, ops = c._keep
                    ops.allgather = rt._ALLGATHER(lambda *a: 1)
                    h = rt.ctypes.c_void_p()
                    rt._check(rt.lib().rt_comm_create_host(rank, world, rt.ctypes.byref(ops), rt.ctypes.byref(h)),
                              "rt_comm_create_host")
                    bad = rt.Comm(h, (cbs, ops))
                    try:
                        bad.selftest(8)
                        q.put((rank, "no error"))
                    except rt.RTError as e:
                        q.put((rank, "raised: " + str(e)))
                    bad.close()
                else:
                    # the healthy ranks' all-gather pairs with nothing: gloo's timeout ends it
                    try:
                        c.selftest(8)
                        q.put((rank, "no error"))
                    except rt.RTError as e:
                        q.put((rank, "raised: " + str(e)))
    finally:
        dist.destroy_process_group()


def _run(world, mode="ok", timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=timeout) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    return out, [p.exitcode for p in ps]


def test_comm_host_world1_needs_no_callback_traffic():
    calls = []

    def never(*a):
        calls.append(a)
        return 1

    ops = rt.CommOps(None, rt._BCAST(never), rt._ALLGATHER(never), rt._SEND(never), rt._RECV(never))
    h = rt.ctypes.c_void_p()
    rt._check(rt.lib().rt_comm_create_host(0, 1, rt.ctypes.byref(ops), rt.ctypes.byref(h)), "rt_comm_create_host")
    c = rt.Comm(h, ops)
    c.selftest(17)
    assert calls == []  # one rank: collectives are local copies
    c.close()


def test_comm_host_rejects_missing_callbacks():
    ops = rt.CommOps()
    h = rt.ctypes.c_void_p()
    assert rt.lib().rt_comm_create_host(0, 2, rt.ctypes.byref(ops), rt.ctypes.byref(h)) == -1


@pytest.mark.parametrize("world", [2, 3])
def test_comm_host_collectives_over_gloo(world):
    out, codes = _run(world)
    assert out == {r: "ok" for r in range(world)}
    assert codes == [0] * world


def test_comm_host_failed_callback_raises():
    """The rank whose all-gather callback fails gets RTError from the library at once."""
    out, _ = _run(2, mode="fail", timeout=200)
    assert out[1].startswith("raised:") and "callback failed" in out[1], out
