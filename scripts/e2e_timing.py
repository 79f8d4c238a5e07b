"""Drop-in GBA call timing on config 4: set_problem + global_ba(10) + the
reads, REPS times (default 3) in one context; SQLM_PREP_TIMING=1 adds the
setup phases on stderr. The last line is the median over reps >= 1 (rep 0
pays the first-touch allocations)."""
import os
import statistics
import sys
import time

sys.path[:0] = ['.', 'sqrtlm-slam_amd']
from sqrtlm import synth
from sqrtlm.optimizer import Context

reps = int(os.environ.get("REPS", "3"))
prob = synth.config4(seed=4)
setup, total = [], []
with Context(0) as ctx:
    for rep in range(reps):
        t0 = time.perf_counter()
        ctx.set_problem(prob)
        t1 = time.perf_counter()
        n, st = ctx.global_ba(10)
        t2 = time.perf_counter()
        ctx.poses(); ctx.points()
        t3 = time.perf_counter()
        print(f"rep {rep}: set_problem {1e3*(t1-t0):.1f} ms, global_ba {1e3*(t2-t1):.1f} (setup {st['ms_setup']:.1f}, lm {st['ms_total']:.1f}, lin {st['ms_linearize']:.1f}), get {1e3*(t3-t2):.1f}", file=sys.stderr, flush=True)
        if rep:
            setup.append(st['ms_setup'])
            total.append(1e3 * (t3 - t0))
if setup:
    print(f"median over reps 1..{reps - 1}: setup {statistics.median(setup):.1f} ms, call {statistics.median(total):.1f} ms",
          file=sys.stderr, flush=True)
