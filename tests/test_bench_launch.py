"""`bench.py --gpus N` without a launcher starts its own N ranks (VERDICT r05
item 1): the driver may run `python3 bench.py --gpus 8` with no torchrun around
it, and that must produce an 8-rank line (or fail), never a 1-GPU line.

CPU tests: the rank environments (--launch-only), the real spawn path with
children that report their environment and exit before importing torch
(--rank-probe), and that one failing rank ends the others and sets the exit
code.  GPU test: two gloo ranks on the box's one GPU run the whole bench and
print an n_gpus = 2 line whose candidates match config D's stock goldens.
"""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
              "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _run(args, timeout=120, env=None):
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env or _env())


def test_launch_only_reports_rank_environments():
    r = _run(["--gpus", "8", "--launch-only"])
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    envs = line["ranks"]
    assert [e["RANK"] for e in envs] == [str(i) for i in range(8)]
    assert [e["LOCAL_RANK"] for e in envs] == [str(i) for i in range(8)]
    assert {e["WORLD_SIZE"] for e in envs} == {"8"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert line["cmd"][1] == BENCH and "--gpus" in line["cmd"]


def test_spawned_ranks_see_torchrun_environment():
    r = _run(["--gpus", "3", "--rank-probe"])
    assert r.returncode == 0, r.stderr
    rows = [json.loads(s) for s in r.stdout.strip().splitlines()]
    assert sorted(int(x["RANK"]) for x in rows) == [0, 1, 2]
    assert {x["WORLD_SIZE"] for x in rows} == {"3"}
    assert {x["MASTER_ADDR"] for x in rows} == {"127.0.0.1"}
    assert len({x["MASTER_PORT"] for x in rows}) == 1
    assert all(x["LOCAL_RANK"] == x["RANK"] for x in rows)


def test_failing_rank_ends_the_others_and_sets_exit_code():
    # rank 1 exits 3 at once; ranks 0 and 2 would sleep 120 s (standing for a
    # rank waiting in a collective): the launcher must end them promptly
    t0 = time.monotonic()
    r = _run(["--gpus", "3", "--rank-probe", "--rank-probe-fail", "1"], timeout=100)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 60


def test_terminating_the_launcher_ends_its_ranks():
    # --rank-probe-fail 9 names no rank: all three ranks sleep (standing for
    # ranks at work), so all are alive when the launcher is stopped
    import signal
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "3", "--rank-probe", "--rank-probe-fail", "9"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=_env())
    seen = 0
    while seen < 3:   # every rank has printed its environment: all started
        line = p.stdout.readline()
        assert line, p.stderr.read()
        seen += 1
    t0 = time.monotonic()
    p.send_signal(signal.SIGTERM)
    rc = p.wait(timeout=60)
    assert rc == 128 + signal.SIGTERM
    assert time.monotonic() - t0 < 40


def test_world_size_mismatch_is_an_error():
    env = _env()
    env.update({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    r = _run(["--gpus", "4", "--rank-probe"], env=env)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_bench_ranks_without_launcher_on_one_gpu(world):
    # gloo: two RCCL ranks cannot share the box's one device
    r = _run(["--gpus", str(world), "--backend", "gloo", "--steps", "2", "--warmup", "1",
              "--no-cpu", "--no-other"], timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == world
    assert line["config"]["parallelism"] == "shard%d" % world
    # every rank's 4 GiB shard against its stock golden (tests/golden/config_d.json)
    assert line["check"]["match_golden"] is True, line["check"]
    assert line["check"]["ascending"] is True
    assert len(line["multi"]["per_rank_step_ms"]["by_rank"]) == world


@pytest.mark.gpu
def test_bench_nccl_ranks_beyond_the_visible_gpus_fail():
    # two RCCL ranks on a one-GPU box: a non-zero exit, never a 1-GPU line
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "1", "--no-cpu", "--no-other"], timeout=300)
    assert r.returncode != 0
    assert not [s for s in r.stdout.splitlines() if s.startswith("{")], r.stdout[-2000:]
