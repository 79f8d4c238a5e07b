"""The persistent cyclic-reduction solve's task graph (k_cr_persist,
cr_persist_graph) against a data-hazard model of launch_cr_core's schedule.

The persistent kernel runs a task as soon as its listed predecessors are
done, in any order the chip picks. That is only the per-level launches'
result if, for every block of data a task reads or writes, every earlier task
(in launch order) that wrote it, and -- for a write -- every earlier task that
read it, is an ancestor through the listed dependencies (RAW, WAW, WAR). The
model below names each task's reads and writes at the granularity the kernels
write them (U / z of a factor, A / C columns, D / E tiles and g slices of an
update, x of a back substitution); the graph comes from tools/cr_graph_dump
(host-only, the same cr_persist_graph the library uploads).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "cr_graph_dump")
F, FO, TR, UP, TOP, BK = range(6)
WORKERS = 12


def _graph(p, n):
    if not os.path.exists(TOOL):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), "cr_graph_dump"], check=True)
    out = subprocess.run([TOOL, str(p), str(n)], check=True, capture_output=True, text=True).stdout
    tasks = []
    for line in out.splitlines():
        head, deps = line.split(":")
        t, I, h, a, b = map(int, head.split())
        tasks.append((t, I, h, a, b, [int(x) for x in deps.split()]))
    return tasks


def _rw(task, p, n):
    """(reads, writes) of one task: sets of hashable data-block names."""
    t, I, h, a, b, _ = task
    nt = n // 16
    nd = nt * (nt + 1) // 2
    R, W = set(), set()
    D = lambda J: {("D", J, k) for k in range(nd)}
    E = lambda J: {("E", J, k) for k in range(nt * nt)}
    G = lambda J: {("g", J, k) for k in range(nt)}
    A = lambda J: {("A", J, k) for k in range(nt)}
    C = lambda J: {("C", J, k) for k in range(nt)}
    if t in (F, FO):
        right = I + h < p
        R |= D(I)
        W.add(("L", I))
        if t == FO:
            R |= G(I)
            W |= G(I)
        else:
            sidx, split = a, b
            fixed = nt - 1  # D columns 1 .. nt-1 (U layout)
            net, nee = nt, (nt if right else 0)
            if sidx != 0:
                W.discard(("L", I))
            for q in range(fixed, WORKERS):
                e = (q - fixed) * split + sidx
                if e < net:
                    R |= E(I - h)
                    W.add(("A", I, e))
                elif e < net + nee:
                    R |= E(I)
                    W.add(("C", I, e - net))
                elif e == net + nee:
                    R |= G(I)
                    W |= G(I)
    elif t == TR:
        right = I + h < p
        R.add(("L", I))
        for s in range(a, a + b):
            if s < nt:
                R |= E(I - h)
                W.add(("A", I, s))
            elif right:
                R |= E(I)
                W.add(("C", I, s - nt))
    elif t == UP:
        J = I
        right, left = J + h < p, J >= h
        for lb in range(a, a + b):
            if lb < nd:
                if right:
                    R |= A(J + h)
                if left:
                    R |= C(J - h)
                if right or left:
                    R.add(("D", J, lb))
                    W.add(("D", J, lb))
            elif lb < nd + nt * nt:
                if right and J + 2 * h < p:
                    R |= A(J + h) | C(J + h)
                    W.add(("E", J, lb - nd))
            else:
                k = lb - nd - nt * nt
                if right:
                    R |= A(J + h) | G(J + h)
                if left:
                    R |= C(J - h) | G(J - h)
                R.add(("g", J, k))
                W.add(("g", J, k))
    elif t == TOP:
        R |= D(0) | G(0)
        W |= {("L", 0), ("x", 0)}
    else:  # BK
        R |= {("L", I), ("x", I - h)} | A(I) | C(I) | G(I)
        if I + h < p:
            R.add(("x", I + h))
        W.add(("x", I))
    return R, W


@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 16, 17, 33, 64, 100, 278])
@pytest.mark.parametrize("n", [48, 112])
def test_persistent_cr_graph_covers_every_hazard(p, n):
    tasks = _graph(p, n)
    anc = []
    last_w, readers = {}, {}
    for i, task in enumerate(tasks):
        deps = task[5]
        assert all(0 <= d < i for d in deps), (i, task)
        a = 0
        for d in deps:
            a |= anc[d] | (1 << d)
        anc.append(a)
        R, W = _rw(task, p, n)
        for x in R:  # read after write
            w = last_w.get(x)
            assert w is None or (a >> w) & 1, ("RAW", p, n, i, task[:5], x, w, tasks[w][:5])
        for x in W:  # write after write / read
            w = last_w.get(x)
            assert w is None or w == i or (a >> w) & 1, ("WAW", p, n, i, task[:5], x, w)
            for r in readers.get(x, ()):
                assert r == i or (a >> r) & 1, ("WAR", p, n, i, task[:5], x, r, tasks[r][:5])
        for x in R:
            readers.setdefault(x, set()).add(i)
        for x in W:
            last_w[x] = i
            readers[x] = set()
    # every superblock's solution is written
    assert {("x", I) for I in range(p)} <= set(last_w)
