import sys, time
sys.path[:0] = ['sqrtlm-slam_amd', '.']
from sqrtlm import synth
from sqrtlm.optimizer import Context
prob = synth.config4(seed=4)
with Context(0) as ctx:
    ctx.set_problem(prob)
    for rep in range(4):
        ms, k, st = ctx.bench(3, 20, True)
        print(round(1000.0 / ms, 1), {a: round(b, 3) for a, b in k.items()}, st.get("trials"), flush=True)
