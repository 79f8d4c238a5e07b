"""A/B of library builds on the default bench (no CPU legs, no extras): value
and the event-timed phase table. usage: python scripts/ab_bench.py lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for lib in sys.argv[1:]:
    env = dict(os.environ, SQLM_LIB_PATH=os.path.join(ROOT, "sqrtlm-slam_amd", "sqrtlm", lib))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-extras",
                          "--steps", "20", "--warmup", "3"], env=env, capture_output=True, text=True, check=True)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    print(lib, round(d["value"], 1), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()}, flush=True)
