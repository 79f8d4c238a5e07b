import sys, time, os
sys.path[:0] = ['.', 'sqrtlm-slam_amd']
from sqrtlm import synth
from sqrtlm.optimizer import Context
prob = synth.config4(seed=4)
with Context(0) as ctx:
    for rep in range(3):
        t0 = time.perf_counter()
        ctx.set_problem(prob)
        t1 = time.perf_counter()
        n, st = ctx.global_ba(10)
        t2 = time.perf_counter()
        ctx.poses(); ctx.points()
        t3 = time.perf_counter()
        print(f"rep {rep}: set_problem {1e3*(t1-t0):.1f} ms, global_ba {1e3*(t2-t1):.1f} (setup {st['ms_setup']:.1f}, lm {st['ms_total']:.1f}, lin {st['ms_linearize']:.1f}), get {1e3*(t3-t2):.1f}", file=sys.stderr, flush=True)
