"""Drop-in LocalBundleAdjustment call timing on config 2: set_problem +
local_ba (three-pass schedule) + the reads, REPS times in one context;
SQLM_PREP_TIMING=1 adds the setup phases of every pass on stderr."""
import os
import statistics
import sys
import time

sys.path[:0] = ['.', 'sqrtlm-slam_amd']
from sqrtlm import synth
from sqrtlm.optimizer import Context

reps = int(os.environ.get("REPS", "5"))
prob = synth.config2()
tot = []
with Context(0) as ctx:
    for rep in range(reps):
        t0 = time.perf_counter()
        ctx.set_problem(prob)
        t1 = time.perf_counter()
        ran, tags, sts = ctx.local_ba()
        t2 = time.perf_counter()
        ctx.poses(); ctx.points()
        t3 = time.perf_counter()
        setup = sum(s['ms_setup'] for s in sts)
        opt = sum(s['ms_total'] for s in sts)
        print(f"rep {rep}: set_problem {1e3*(t1-t0):.2f} ms, local_ba {1e3*(t2-t1):.2f} (setup {setup:.2f}, lm {opt:.2f}, "
              f"passes {len(sts)}), get {1e3*(t3-t2):.2f}, call {1e3*(t3-t0):.2f}", file=sys.stderr, flush=True)
        if rep:
            tot.append(1e3 * (t3 - t0))
if tot:
    print(f"median call over reps 1..{reps - 1}: {statistics.median(tot):.2f} ms", file=sys.stderr, flush=True)
