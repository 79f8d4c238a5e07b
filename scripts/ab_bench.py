"""A/B of library builds on the default bench (no CPU legs, no extras): value
and the event-timed phase table. usage: python scripts/ab_bench.py lib1.so lib2.so ...
(AB_ARGS="--config lba" passes bench arguments; a lib written NAME.so:VAR=1
runs NAME.so with that environment variable set)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
extra = os.environ.get("AB_ARGS", "").split()
for spec in sys.argv[1:]:
    lib, *var = spec.split(":")
    env = dict(os.environ, SQLM_LIB_PATH=os.path.join(ROOT, "sqrtlm-slam_amd", "sqrtlm", lib))
    for v in var:
        k, _, x = v.partition("=")
        env[k] = x
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-extras",
                          "--steps", "20", "--warmup", "3"] + extra, env=env, capture_output=True, text=True,
                         check=True)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    e2e = d.get("end_to_end") or {}
    print(spec, round(d["value"], 1), {k: round(v, 4) for k, v in d["kernel_ms_per_step"].items()},
          "e2e_ms %.2f" % (1e3 * e2e["seconds"]) if "seconds" in e2e else "", flush=True)
