"""Device bounds checks (SURVEY.md §5 "device bounds asserts in a debug build"; kernels.h
L3_DCHECK): the check build of the library (libllama3hip_check.so — the same sources with
-DL3_DEVICE_CHECKS, counters instead of traps) runs every kernel family to the last cache slot
with no violation recorded, and its self-test shows the counters reach the host; the release
library reports the checks compiled out."""
import json
import os
import subprocess
import sys

import pytest

import l3hip

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CHECK_LIB = os.path.join(os.path.dirname(HERE), "llama3.np_amd", "csrc", "libllama3hip_check.so")


def test_release_library_has_no_device_checks():
    ctx = l3hip.op_context(0)
    enabled, counts = ctx.device_check_counts()
    ctx.device_check_selftest()  # a no-op here
    assert not enabled and counts == {"kv_slot": 0, "attn_keys": 0, "token_id": 0}
    assert ctx.device_check_counts()[1] == counts


def test_check_build_records_no_violation():
    if not os.path.exists(CHECK_LIB):
        pytest.skip(f"{CHECK_LIB} missing: build it with `make -C llama3.np_amd/csrc check-lib` "
                    "(__graft_entry__.build() does)")
    env = dict(os.environ, L3_LIB_PATH=CHECK_LIB)
    r = subprocess.run([sys.executable, os.path.join(HERE, "device_checks_workload.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["enabled"] is True
    assert out["selftest"] == {"kv_slot": 1, "attn_keys": 1, "token_id": 1}
    assert out["after_selftest_read"] == {"kv_slot": 0, "attn_keys": 0, "token_id": 0}
    assert out["workload"] == {"kv_slot": 0, "attn_keys": 0, "token_id": 0}
    assert out["persistent"] is True
