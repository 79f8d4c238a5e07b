"""Launch schedules against each other, bit for bit: the pose update folded
into the first landmark-update launch (default for small problems) vs its own
launch (SQLM_NO_POSE_FUSE=1). It replaces a launch only -- the arithmetic is
the same device code in the same order -- so poses, points, edge chi2,
outlier tags and the whole LM trace must be equal (==), on the problems of
test_gpu_spec.py (including rejected trials and the three-pass local-BA
schedule).
"""
import numpy as np
import pytest

from test_gpu_spec import CASES, _strip

pytestmark = pytest.mark.gpu


def _run(ctx, prob, kind, monkeypatch, env):
    for k, v in env.items():
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, v)
    ctx.set_problem(prob)
    if kind == "global":
        out = ctx.global_ba(12)
    elif kind == "local":
        ran, tags, sts = ctx.local_ba()
        out = (ran, tags.tolist(), sts)
    else:
        out = ctx.optimize(0, 20)
    q, t = ctx.poses()
    info = ctx.exec_info()
    return out, q.copy(), t.copy(), ctx.points().copy(), ctx.edge_chi2().copy(), info


NEW = {"SQLM_NO_POSE_FUSE": None}
OLD = {
    "pose_launch": {"SQLM_NO_POSE_FUSE": "1"},
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("old", sorted(OLD))
def test_schedule_bitwise_equal(gpu_ctx, monkeypatch, name, old):
    kind, make = CASES[name]
    prob = make()
    a = _run(gpu_ctx, prob, kind, monkeypatch, NEW)
    b = _run(gpu_ctx, prob, kind, monkeypatch, {**NEW, **OLD[old]})
    if kind == "local":
        assert a[0][0] == b[0][0] and a[0][1] == b[0][1]
        assert _strip(a[0][2]) == _strip(b[0][2])
    else:
        assert a[0][0] == b[0][0]
        assert _strip(a[0][1]) == _strip(b[0][1])
    for x, y in zip(a[1:5], b[1:5]):
        assert np.array_equal(x, y)
