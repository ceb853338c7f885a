"""Multi-GPU host logic on CPU: the N > 1 bench line's device proof (bench.check_devices) and
the single-process group's row mapping (l3hip.member_rows, the l3_group_* C ABI's mapping).

The reference never mixes batch rows (llama3.py:163-211), so the batch axis shards; these pin
the parts of the sharded path that need no GPU.  The device paths run in tests/test_gpu_parity.py
(world 1 on the one-GPU box) and in the driver's 8-GPU scaling run.
"""

import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import l3hip  # noqa: E402

BUS = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xe5, 0xf5)]


def test_check_devices_fields():
    out = bench.check_devices(8, 8, BUS, 3, 3)
    assert out == {"rccl_nranks": 8, "devices": BUS}


@pytest.mark.parametrize("case", ["duplicate", "count", "rank", "short_list"])
def test_check_devices_refuses(case, capsys):
    n, world, bus, seen, rank = 8, 8, list(BUS), 2, 2
    if case == "duplicate":  # two ranks on one GPU (e.g. LOCAL_RANK ignored)
        bus[5] = bus[2]
    elif case == "count":  # RCCL formed a smaller communicator than WORLD_SIZE
        n, bus = 4, bus[:4]
    elif case == "rank":
        seen = 5
    else:
        bus = bus[:7]
    with pytest.raises(SystemExit) as e:
        bench.check_devices(n, world, bus, seen, rank)
    assert e.value.code == 4
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["error"] == "multi-GPU device check failed" and line["details"]


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_member_rows_interleave(n):
    for B in range(0, 70):
        counts = [l3hip.member_rows(B, n, i) for i in range(n)]
        assert sum(counts) == B
        assert max(counts) - min(counts) <= 1
        # row r = i + n * j for j < counts[i]: every row once, local index r // n
        seen = sorted(i + n * j for i in range(n) for j in range(counts[i]))
        assert seen == list(range(B))
        assert all(counts[r % n] > r // n for r in range(B))
    # the mapping does not depend on B: row r's member and local row are the same in every batch
    for r in range(40):
        owners = {(r % n, r // n) for B in range(r + 1, 60)}
        assert len(owners) == 1


def test_member_rows_bad_member():
    with pytest.raises(ValueError):
        l3hip.member_rows(8, 2, 2)
