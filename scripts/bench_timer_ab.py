"""GPU-box helper: the config-4 bench iterations repeated, with and without
the per-phase timing events, on one context and on fresh contexts, to
separate the timer cost from run-to-run drift."""
import sys
import time

sys.path[:0] = ['sqrtlm-slam_amd', '.']
from sqrtlm import synth  # noqa: E402
from sqrtlm.optimizer import Context  # noqa: E402

prob = synth.config4(seed=4)
mode = sys.argv[1] if len(sys.argv) > 1 else "same"
t0 = time.time()
if mode == "same":
    with Context(0) as ctx:
        ctx.set_problem(prob)
        for rep in range(3):
            for timers in (False, True):
                ms, k, st = ctx.bench(3, 20, timers)
                print(f"{time.time() - t0:6.1f}s", "timers" if timers else "plain ", round(1000.0 / ms, 1), flush=True)
else:
    for rep in range(3):
        for timers in (False, True):
            with Context(0) as ctx:
                ctx.set_problem(prob)
                ms, k, st = ctx.bench(3, 20, timers)
            print(f"{time.time() - t0:6.1f}s", "fresh", "timers" if timers else "plain ", round(1000.0 / ms, 1),
                  flush=True)
