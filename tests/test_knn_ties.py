"""The oracle's photon kNN (myKD_Tree.find_near, myLight.java:389-445) breaks exact distance ties as
the reference does: its max-queue is java.util.PriorityQueue with Collections.reverseOrder(), whose
JDK 8 sifts (siftUpUsingComparator / siftDownUsingComparator) decide which of several equally
distant photons poll() evicts once the queue holds num_near, and the poll order of the sum.

The expected neighbourhoods come from a small independent restatement here: the kd-tree build
(build_tree :332-381, Collections.sort is stable like Python's sort), the recursive search, and
JDK 8's PriorityQueue.offer / poll. Photons sit on an integer lattice with duplicated points, so
whole shells of photons share a distance and every neighbourhood boundary is a tie."""
import numpy as np
import pytest

from oracle.oracle import OracleScene


# ---- java.util.PriorityQueue (JDK 8) with a reversed comparator on d2: a max-heap
def pq_add(q, e):  # offer -> siftUpUsingComparator
    k = len(q)
    q.append(e)
    while k > 0:
        parent = (k - 1) >> 1
        if q[parent][0] >= e[0]:  # reverseOrder.compare(x, parent) >= 0
            break
        q[k] = q[parent]
        k = parent
    q[k] = e


def pq_poll(q):  # poll -> siftDownUsingComparator(0, last)
    r = q[0]
    x = q.pop()
    n = len(q)
    if n > 0:
        k, half = 0, n >> 1
        while k < half:
            child = 2 * k + 1
            if child + 1 < n and q[child + 1][0] > q[child][0]:
                child += 1
            if x[0] >= q[child][0]:
                break
            q[k] = q[child]
            k = child
        q[k] = x
    return r


# ---- myKD_Tree
def build(pl):  # build_tree on a list of (pos[3], id)
    if len(pl) == 1:
        return (pl[0], -1, None, None)
    mins = [1e20] * 3
    maxs = [-1e20] * 3
    for p, _ in pl:
        for j in range(3):
            mins[j] = min(mins[j], p[j]) if p[j] < mins[j] else mins[j]
            maxs[j] = p[j] if p[j] > maxs[j] else maxs[j]
    dx, dy, dz = maxs[0] - mins[0], maxs[1] - mins[1], maxs[2] - mins[2]
    ax = 0 if (dx >= dy and dx >= dz) else 1 if (dy >= dx and dy >= dz) else 2
    pl = sorted(pl, key=lambda e: e[0][ax])  # Collections.sort: stable
    sp = len(pl) // 2
    left = build(pl[:sp]) if sp != 0 else None
    right = build(pl[sp + 1:]) if sp != len(pl) - 1 else None
    return (pl[sp], ax, left, right)


def find_near(root, pos, k, max_d2):
    q = []
    state = {"m": max_d2}

    def rec(node):
        (ph, pid), ax, left, right = node
        if ax != -1:
            delta = pos[ax] - ph[ax]
            d2 = delta * delta
            if delta < 0:
                if left is not None:
                    rec(left)
                if right is not None and d2 < state["m"]:
                    rec(right)
            else:
                if right is not None:
                    rec(right)
                if left is not None and d2 < state["m"]:
                    rec(left)
        dx, dy, dz = pos[0] - ph[0], pos[1] - ph[1], pos[2] - ph[2]
        len2 = dx * dx + dy * dy + dz * dz
        if len2 < state["m"]:
            pq_add(q, (len2, pid))
            if len(q) > k:
                pq_poll(q)
            if len(q) == k and q[0][0] < state["m"]:
                state["m"] = q[0][0]

    rec(root)
    out = []
    while q:
        out.append(pq_poll(q))
    return out


def _lattice(seed):
    rng = np.random.default_rng(seed)
    g = np.stack(np.meshgrid(np.arange(-3, 4), np.arange(-3, 4), np.arange(-1, 2), indexing="ij"), -1).reshape(-1, 3)
    pos = np.concatenate([g, g[rng.choice(len(g), 40, replace=False)]]).astype(np.float64)  # duplicated points
    pos = pos[rng.permutation(len(pos))]
    pwr = rng.random((len(pos), 3))
    return pos, pwr


@pytest.mark.parametrize("k", [5, 6, 13, 30])
@pytest.mark.parametrize("seed", [1, 2])
def test_knn_ties_follow_java_priority_queue(tmp_path, k, seed):
    cli = tmp_path / "knn.cli"
    cli.write_text(f"fov 60\nbackground 0 0 0\npoint_light 0 5 0 1 1 1\ndiffuse_photons 100 {k} 10\n"
                   "diffuse .5 .5 .5 0 0 0\nsphere 1 0 0 -5\n")
    pos, pwr = _lattice(seed)
    o = OracleScene(tmp_path, "knn.cli")
    o.set_photons(pos, pwr)
    root = build([(tuple(p), i) for i, p in enumerate(pos.tolist())])
    queries = [(0.0, 0.0, 0.0), (0.5, 0.0, 0.0), (0.5, 0.5, 0.0), (1.0, -1.0, 0.5), (-2.0, 1.0, 0.0)]
    ties = 0
    for qp in queries:
        exp = find_near(root, qp, k, 100.0)
        idx, d2 = o.knn(qp)
        assert [i for _, i in exp] == idx.tolist(), (qp, exp, idx)
        assert [d for d, _ in exp] == d2.tolist()
        ties += len(set(d for d, _ in exp)) < len(exp)
    assert ties == len(queries)  # every neighbourhood holds equally distant photons


def _flatten(node, out):  # the Python build_tree's nodes in DFS pre-order: (photon id, axis, left, right)
    me = len(out)
    (_, pid), ax, left, right = node
    out.append([pid, ax, -1, -1])
    if left is not None:
        out[me][2] = len(out)
        _flatten(left, out)
    if right is not None:
        out[me][3] = len(out)
        _flatten(right, out)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_product_kdtree_is_the_references(seed):
    """The product's copy of myKD_Tree.build_tree (csrc/photon.cpp, the structure the device's tie
    replay walks; host-only rt_photon_kdtree) equals the independent Python restatement node for
    node -- on the duplicated lattice (every stable-sort tie decided by the previous order) and on
    random photons large enough for the parallel subtree builds and the merge sort."""
    from distraytracer_old_amd import rt

    pos, _ = _lattice(seed)
    rng = np.random.default_rng(seed)
    big = np.concatenate([rng.random((9000, 3)), np.round(rng.random((3000, 3)) * 8) / 8])  # ties too
    big[rng.random(len(big)) < 0.05, 1] = -0.0
    for p in (pos, big):
        exp = np.array(_flatten(build([(tuple(q), i) for i, q in enumerate(p.tolist())]), []), dtype=np.int32)
        got = rt.photon_kdtree(p)
        assert np.array_equal(got, exp)
