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



def _rccl_rank(rank, world, port, mode, q):
    """One gloo rank of connect_rccl with a stand-in context whose
    set_comm / comm_info behave as `mode` says."""
    import torch.distributed as dist
    from sqrtlm._lib import SqlmError
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class FakeCtx:
        def set_comm(self, uid, r, n):
            self.uid = uid
            if mode == "fail" and r == 1:
                raise SqlmError(-9, "sqlm_ctx_set_comm")

        def comm_info(self):
            n = world - 1 if mode == "short" else world
            return {"transport": "rccl", "rank": rank, "nranks": n}

    ctx = FakeCtx()
    try:
        res = bench.connect_rccl(ctx, rank, world, dist, lambda: bytes(range(7, 135)))
        q.put((rank, "ok", res, ctx.uid == bytes(range(7, 135))))
    except SystemExit as e:
        q.put((rank, "exit", e.code, None))
    dist.destroy_process_group()


def _run_rccl(mode, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=_rccl_rank, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    return out


def test_rccl_init_failure_exits_nonzero_on_every_rank():
    """A communicator that fails on one rank ends EVERY rank with a non-zero
    status (no silent switch to the host transport, bench.py writes no line)."""
    out = _run_rccl("fail")
    assert [o[1] for o in out] == ["exit", "exit"], out
    assert {o[2] for o in out} == {bench.CommInitFailed.STATUS} and bench.CommInitFailed.STATUS != 0


def test_rccl_rank_count_mismatch_exits_nonzero():
    """ncclCommCount disagreeing with WORLD_SIZE is a failure too."""
    out = _run_rccl("short")
    assert [o[1] for o in out] == ["exit", "exit"], out


def test_rccl_success_reports_communicator_ranks():
    out = _run_rccl("ok", world=3)
    assert [o[1] for o in out] == ["ok"] * 3, out
    for _r, _s, (desc, n), same_uid in out:
        assert n == 3 and "3 ranks reported by ncclCommCount" in desc and same_uid
