"""A/B: the same GBA on two library builds must give bitwise-equal results
(a kernel change that keeps every summation order). usage:
python scripts/ab_bits.py libsqrtlm_old.so[:VAR=V...] [scale]
(the A side may carry environment settings, e.g. libsqrtlm.so:SQLM_TILE_PROD=0
compares the in-tree library against itself with that switch)"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(spec, scale, out):
    lib, *var = spec.split(":") if spec else ("",)
    env = dict(os.environ, SQLM_LIB_PATH=os.path.join(ROOT, "sqrtlm-slam_amd", "sqrtlm", lib) if lib else "")
    if not lib:
        env.pop("SQLM_LIB_PATH")
    for v in var:
        k, _, x = v.partition("=")
        env[k] = x
    code = f"""
import sys; sys.path.insert(0, {os.path.join(ROOT, 'sqrtlm-slam_amd')!r})
import numpy as np
from sqrtlm import synth
from sqrtlm.optimizer import Context
for gen in ("band", "loop", "lba"):
    with Context(0) as c:
        if gen == "lba":  # config 2 through the three-pass local-BA schedule (small-problem paths)
            c.set_problem(synth.config2()); ran, tags, sts = c.local_ba(); st = sts[-1]
        else:
            p = synth.config4(seed=4, scale={scale}) if gen == "band" else synth.config4_loop(seed=4, scale={scale})
            c.set_problem(p); n, st = c.global_ba(5)
        q, t = c.poses()
        np.savez({out!r} + gen, q=q, t=t, X=c.points(), chi=np.array(st["trace_chi2"]))
"""
    subprocess.run([sys.executable, "-c", code], env=env, check=True)


scale = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
run(sys.argv[1], scale, "/tmp/ab_a_")
run("", scale, "/tmp/ab_b_")
for gen in ("band", "loop", "lba"):
    a, b = np.load(f"/tmp/ab_a_{gen}.npz"), np.load(f"/tmp/ab_b_{gen}.npz")
    same = all(np.array_equal(a[k], b[k]) for k in ("q", "t", "X", "chi"))
    print(gen, "bitwise equal" if same else f"DIFFER max dq {np.abs(a['q'] - b['q']).max():.3e} chi {a['chi'][-1]} {b['chi'][-1]}")
