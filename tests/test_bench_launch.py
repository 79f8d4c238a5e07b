"""bench.py's N>1 launch contract (CPU, no GPU touched):

* `--gpus N` without a launcher starts the N ranks itself (RANK / LOCAL_RANK /
  WORLD_SIZE / MASTER_* as torch.distributed.run sets them) and exits with
  their worst status;
* `--gpus N` under a launcher whose WORLD_SIZE differs exits non-zero before
  doing anything, so a line can never claim n_gpus it did not run on.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _bench(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus_world_size_mismatch_fails():
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr
    assert "--gpus 2" in r.stderr and "WORLD_SIZE=1" in r.stderr
    r = _bench(["--gpus", "1"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr


def test_gpus_must_be_positive():
    r = _bench(["--gpus", "0"], {})
    assert r.returncode == 2 and "must be >= 1" in r.stderr


def test_spawn_ranks_environment(tmp_path):
    """Every rank sees its own RANK / LOCAL_RANK, the common WORLD_SIZE and one
    rendezvous address on 127.0.0.1."""
    out = tmp_path / "r{}.json"
    code = ("import json, os; r = os.environ['RANK']; "
            f"open(r'{out}'.format(r), 'w').write(json.dumps({{k: os.environ[k] for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}))")
    assert bench.spawn_ranks(3, [sys.executable, "-c", code]) == 0
    seen = [json.loads(open(str(out).format(r)).read()) for r in range(3)]
    assert [s["RANK"] for s in seen] == ["0", "1", "2"]
    assert [s["LOCAL_RANK"] for s in seen] == ["0", "1", "2"]
    assert {s["WORLD_SIZE"] for s in seen} == {"3"} and {s["LOCAL_WORLD_SIZE"] for s in seen} == {"3"}
    assert {s["MASTER_ADDR"] for s in seen} == {"127.0.0.1"} and len({s["MASTER_PORT"] for s in seen}) == 1


def test_spawn_ranks_failure_ends_the_job():
    """A rank that fails makes the job fail, and the ranks still waiting for it
    (a collective that can never complete) are ended, not left hanging."""
    code = ("import os, sys, time; r = int(os.environ['RANK']); "
            "sys.exit(3) if r == 1 else time.sleep(60)")
    t0 = __import__("time").time()
    assert bench.spawn_ranks(3, [sys.executable, "-c", code]) != 0
    assert __import__("time").time() - t0 < 30

