"""bench.py's launcher-free multi-GPU path (spawn_ranks), on CPU with a stub rank body.

`python bench.py --gpus N` without torch.distributed.run must start N fresh rank processes
itself (one per GPU, the reference's rows are independent: llama3.py:163-211), hand each the
torchrun environment and a launch key unique to the launch, forward rank 0's stdout, and exit
with a failing rank's status.  The stub stands in for the GPU rank body: it records its
environment and exits with the code the test asks of it.
"""

import io
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

STUB = r"""
import json, os, sys, time
out, fail_rank, rc, sleep_rank = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
r = int(os.environ["RANK"])
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "L3_LAUNCH_KEY")
with open(os.path.join(out, f"rank{r}.json"), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys} | {"ppid": os.getppid()}, f)
if r == 0:
    print(json.dumps({"metric": "stub", "rank": r}), flush=True)
if r == sleep_rank:
    time.sleep(600)  # a peer stuck in a collective: must be killed by the parent
sys.exit(rc if r == fail_rank else 0)
"""


def _run(tmp_path, n, fail_rank=-1, rc=0, sleep_rank=-1, grace_s=20.0, timeout_s=120):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    out = tmp_path / "out"
    out.mkdir(exist_ok=True)
    log = tmp_path / "stdout.txt"
    with open(log, "w") as f:
        status = bench.spawn_ranks(n, [str(out), str(fail_rank), str(rc), str(sleep_rank)],
                                   cmd=[sys.executable, str(stub)], timeout_s=timeout_s, grace_s=grace_s,
                                   out=f)
    envs = {}
    for p in out.iterdir():
        with open(p) as f:
            e = json.load(f)
        envs[int(e["RANK"])] = e
    return status, envs, log.read_text()


def test_spawn_env_and_rank0_line(tmp_path):
    status, envs, stdout = _run(tmp_path, 4)
    assert status == 0
    assert sorted(envs) == [0, 1, 2, 3]
    ports = {e["MASTER_PORT"] for e in envs.values()}
    keys = {e["L3_LAUNCH_KEY"] for e in envs.values()}
    assert len(ports) == 1 and len(keys) == 1  # one launch: every rank agrees
    for r, e in envs.items():
        assert e["LOCAL_RANK"] == str(r) and e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert e["ppid"] == os.getpid()  # children of this process (spawned, not exec'd)
    # only rank 0 writes the forwarded stdout: exactly its one JSON line
    lines = [x for x in stdout.splitlines() if x.strip()]
    assert lines == [json.dumps({"metric": "stub", "rank": 0})]


def test_spawn_launch_keys_unique(tmp_path):
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    a = _run(tmp_path / "a", 2)[1]
    b = _run(tmp_path / "b", 2)[1]
    assert a[0]["L3_LAUNCH_KEY"] != b[0]["L3_LAUNCH_KEY"]


def test_launch_key_honours_env(monkeypatch):
    import l3hip

    monkeypatch.setenv("L3_LAUNCH_KEY", "spawn_x_1_abc")
    assert l3hip.launch_key() == "spawn_x_1_abc"
    monkeypatch.delenv("L3_LAUNCH_KEY")
    monkeypatch.setenv("MASTER_PORT", "4242")
    assert l3hip.launch_key().endswith("_4242")


def test_spawn_failing_rank_status(tmp_path):
    status, envs, _ = _run(tmp_path, 3, fail_rank=2, rc=3)
    assert status == 3 and sorted(envs) == [0, 1, 2]


def test_spawn_kills_peers_of_a_failed_rank(tmp_path):
    # rank 1 fails at once, rank 2 hangs (as a peer blocked in RCCL would): the parent kills it
    # after the grace period and reports rank 1's status
    status, envs, _ = _run(tmp_path, 3, fail_rank=1, rc=5, sleep_rank=2, grace_s=1.0)
    assert status == 5 and sorted(envs) == [0, 1, 2]


def test_spawn_timeout_kills_hung_launch(tmp_path):
    # no rank fails but one never returns (every rank stuck in RCCL init looks like this): the
    # launch-wide timeout kills it and reports 124; the finally reaps every child
    import time

    t0 = time.time()
    status, envs, _ = _run(tmp_path, 2, sleep_rank=1, timeout_s=2.0)
    assert status == 124 and sorted(envs) == [0, 1]
    assert time.time() - t0 < 60


def test_bench_cli_spawns_without_world_size(tmp_path):
    """The real entry point: `python bench.py --gpus 2` with no WORLD_SIZE starts two ranks
    (each of which, here without a GPU library call, stops at argument checks: --workload
    with an impossible --global-batch makes every rank exit 2 before touching the GPU)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--global-batch", "3"], env=env, capture_output=True, text=True, timeout=300)
    # each rank: "--global-batch 3 not divisible by 2 GPUs" -> SystemExit(msg) -> status 1
    assert p.returncode == 1, p.stderr
    assert "not divisible by 2" in p.stderr
    assert '"rank failed"' in p.stderr
