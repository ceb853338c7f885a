"""The C ABI driven from a plain C host (tests/c_api_smoke.c), on the GPU.

``c_smoke`` links libllama3hip.so; ``c_smoke_asan`` links a build of the same sources with
host-side AddressSanitizer (sanitizers on host code; the gfx950 code
objects are unchanged).  Both are built in-tree by ``make -C llama3.np_amd/csrc``.
"""

import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llama3.np_amd", "csrc")


@pytest.mark.parametrize("binary", ["c_smoke", "c_smoke_asan"])
def test_c_host_smoke(binary):
    exe = os.path.join(CSRC, binary)
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make -C llama3.np_amd/csrc)")
    env = dict(os.environ)
    # the HIP runtime's own allocations are not ours to audit at exit
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, f"rc={r.returncode}\nstdout:\n{r.stdout}\nstderr:\n{r.stderr[-4000:]}"
    assert "c_api_smoke ok" in r.stdout
    assert "AddressSanitizer" not in r.stderr
