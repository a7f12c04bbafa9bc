"""``bench.py --gpus N``: the rank launcher and the N-rank aggregation, on CPU (gloo).

The driver's scaling run either starts the ranks itself (torchrun) or calls
``bench.py --gpus N``; both must give one rank per distinct GPU (reference data
parallelism: one process per device, shards ``i % world == rank``,
hpc_source.py:154-156, seed + rank, config.py:204) and a line whose ``value`` is the
whole job's images over the slowest rank's time.  ``--dry-run`` runs the same
launcher, env, gloo group and rank-0 report without GPU work.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

ENV_KEYS = ["RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ENV_KEYS}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=str(ROOT))


def test_launcher_gives_each_worker_its_rank(capfd):
    probe = [sys.executable, "-c",
             "import os, json; print(json.dumps({k: os.environ.get(k) for k in %r}), flush=True)" % ENV_KEYS]
    rc = bench.launch_ranks(2, [], devices=2, cmd=probe)
    assert rc == 0
    lines = [json.loads(x) for x in capfd.readouterr().out.strip().splitlines()]
    assert sorted(int(d["RANK"]) for d in lines) == [0, 1]
    for d in lines:
        assert d["WORLD_SIZE"] == "2" and d["LOCAL_RANK"] == d["RANK"] and d["LOCAL_WORLD_SIZE"] == "2"
        assert d["MASTER_ADDR"] == "127.0.0.1" and int(d["MASTER_PORT"]) > 0
    assert len({d["MASTER_PORT"] for d in lines}) == 1


def test_launcher_refuses_too_few_devices():
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.launch_ranks(8, [], devices=1)
    with pytest.raises(SystemExit, match="no GPU"):
        bench.check_devices(1, 0, rehearsal=True)
    bench.check_devices(8, 1, rehearsal=True)  # explicit rehearsal: allowed


def test_launcher_propagates_a_failing_rank():
    cmd = [sys.executable, "-c", "import os, sys, time; r = int(os.environ['RANK']); "
                                 "sys.exit(3) if r == 1 else time.sleep(60)"]
    assert bench.launch_ranks(2, [], devices=2, cmd=cmd) == 3  # rank 0 is terminated, not waited for


def test_dry_run_two_ranks_aggregates_over_gloo():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "4", "--batch", "8"], {"DINO_BENCH_DEVICES": "2"})
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["ranks"] == 2 and line["n_gpus"] == 2 and "rehearsal" not in line
    assert [p["rank"] for p in line["per_rank"]] == [0, 1]
    assert [p["device"] for p in line["per_rank"]] == [0, 1]
    # value = all ranks' images / the slowest rank's time (rank 1's fake time is 10 % longer)
    slow = max(p["ms_per_step"] for p in line["per_rank"])
    assert line["ms_per_step"] == pytest.approx(slow)
    assert line["value"] == pytest.approx(2 * 8 / (slow / 1e3), rel=1e-3)


def test_dry_run_refuses_shared_devices_unless_rehearsal():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "2"], {"DINO_BENCH_DEVICES": "1"})
    assert r.returncode != 0 and "only 1 GPU" in r.stderr
    r = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--rehearsal"], {"DINO_BENCH_DEVICES": "1"})
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["rehearsal"] is True and line["n_gpus"] == 1 and line["ranks"] == 2


def test_rank_count_must_match_gpus_flag():
    r = _run(["--gpus", "3", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0",
                                             "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29999"})
    assert r.returncode != 0 and "--gpus 3" in r.stderr


@pytest.mark.parametrize("leg", ["c2_prog", "e2e"])
def test_host_fed_legs_run_in_a_child_process(monkeypatch, leg):
    """The c2_prog and (N = 1) e2e legs run as ``bench.py --only-leg <leg>`` children with
    the parent's data sizes and seeds (one loader pipeline per process, as in training;
    DESIGN.md §5), without the parent's rank environment; a failing child fails the leg."""
    args = bench.build_parser().parse_args(["--steps", "7", "--warmup", "2", "--batch", "64", "--unique", "32",
                                            "--mixed", "--gather-threads", "3"])
    seen = {}

    class _Done:
        returncode = 0
        stdout = json.dumps({"value": 1.0}) + "\n"
        stderr = ""

    def fake_run(cmd, **kw):
        seen["cmd"], seen["env"] = cmd, kw.get("env", {})
        return _Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setenv("RANK", "0")
    res = bench.run_leg_child(args, leg)
    cmd = seen["cmd"]
    assert cmd[1].endswith("bench.py") and cmd[cmd.index("--only-leg") + 1] == leg
    for flag, val in (("--steps", "7"), ("--warmup", "2"), ("--batch", "64"), ("--unique", "32"),
                      ("--gather-threads", "3")):
        assert cmd[cmd.index(flag) + 1] == val
    assert "--mixed" in cmd and "RANK" not in seen["env"]
    assert res["value"] == 1.0 and res["process"].startswith("child")

    class _Fail(_Done):
        returncode = 3
        stderr = "boom"

    monkeypatch.setattr(subprocess, "run", lambda cmd, **kw: _Fail())
    with pytest.raises(RuntimeError, match="boom"):
        bench.run_leg_child(args, leg)
