set -o pipefail
SQLM_PREP_TIMING=1 timeout -k 10 300 python3 -c "
import sys, time; sys.path[:0]=['sqrtlm-slam_amd','.']
from sqrtlm import synth
from sqrtlm.optimizer import Context
p = synth.config4(seed=4)
with Context(0) as ctx:
    for r in range(2):
        t=time.perf_counter(); ctx.set_problem(p); n, st = ctx.global_ba(10); print('e2e', time.perf_counter()-t, st['ms_setup'], st['ms_total'], flush=True)
"
