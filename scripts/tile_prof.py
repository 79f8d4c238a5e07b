"""Phase breakdown of k_rcs_tile from the diagnostic library build
(make -C sqrtlm-slam_amd/csrc PROF=1): cycles per phase summed over the
first 64 tiles and all launches, as fractions of the batch loop."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SQLM_LIB_PATH"] = os.path.join(ROOT, "sqrtlm-slam_amd", "sqrtlm", "libsqrtlm_prof.so")
sys.path.insert(0, os.path.join(ROOT, "sqrtlm-slam_amd"))
import numpy as np  # noqa: E402
from sqrtlm import synth  # noqa: E402
from sqrtlm._lib import lib  # noqa: E402
from sqrtlm.optimizer import Context  # noqa: E402

prob = synth.config4(seed=4, scale=float(sys.argv[1]) if len(sys.argv) > 1 else 1.0)
with Context(0) as ctx:
    ctx.set_problem(prob)
    ms, kms, st = ctx.bench(0, 2)
    prof = np.zeros((64, 8), np.int64)
    assert lib().sqlm_debug_tile_profile(prof.ctypes.data_as(C.c_void_p)) == 0
if os.environ.get("SQLM_TILE_PROD", "1") != "0":
    # k_rcs_tile_p: producer (wave 0) and first consumer (wave 1), each as
    # fractions of its own time
    prod, cons = prof[:, 0:2].sum(), prof[:, 2:4].sum()
    print(json.dumps({"ms_per_iter": ms, "k_rcs_tile_ms": kms["k_rcs_tile"], "kernel": "k_rcs_tile_p",
                      "producer": {"stage": round(float(prof[:, 0].sum()) / prod, 4),
                                   "wait": round(float(prof[:, 1].sum()) / prod, 4)},
                      "consumer": {"mfma+grad": round(float(prof[:, 2].sum()) / cons, 4),
                                   "wait": round(float(prof[:, 3].sum()) / cons, 4)},
                      "cycles_per_tile_per_launch": float(prod) / 64 / 2}))
else:
    names = ["stage", "barrierA", "fetch_issue", "clear", "mfma", "g+range", "barrierB", "-"]
    tot = prof[:, :7].sum()
    print(json.dumps({"ms_per_iter": ms, "k_rcs_tile_ms": kms["k_rcs_tile"],
                      "phase_frac": {n: round(float(prof[:, i].sum()) / tot, 4) for i, n in enumerate(names[:7])},
                      "cycles_per_tile_per_launch": float(tot) / 64 / 2}))
