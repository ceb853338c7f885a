"""The C-ABI library loads on a CPU-only host and exports every symbol the header declares.

No compute entry point is called here (there is no GPU in the build container).
"""

import ctypes
import os
import re
import subprocess

import pytest

import l3hip


def test_library_exports_every_header_symbol():
    lib = l3hip.lib()
    declared = l3hip.header_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, f"declared in include/llama3hip.h but not exported: {missing}"


def test_binding_signatures_cover_header():
    declared = set(l3hip.header_symbols())
    bound = set(l3hip._SIGNATURES)
    assert declared == bound, (declared - bound, bound - declared)


def test_exports_are_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", l3hip.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in l3hip.header_symbols():
        assert s in exported, s  # unmangled: extern "C"


def test_code_object_targets_gfx950_only():
    with open(l3hip.LIB_PATH, "rb") as f:
        blob = f.read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx\w+)", blob))
    assert targets == {b"gfx950"}, targets


def test_error_path_without_device_is_loud():
    """A compute call with a null context returns an error and sets a message."""
    lib = l3hip.lib()
    rc = lib.l3_synchronize(None)
    assert rc != 0
    assert b"null context" in lib.l3_last_error()
    with pytest.raises(RuntimeError, match="null context"):
        l3hip.check(lib.l3_finalize(None))


def test_dims_struct_layout():
    assert ctypes.sizeof(l3hip.Dims) == 9 * 4


def test_library_path_is_in_tree():
    assert os.path.dirname(l3hip.LIB_PATH).endswith(os.path.join("llama3.np_amd", "csrc"))


@pytest.mark.parametrize("kw,msg", [
    (dict(dim=320, n_heads=4, n_kv_heads=4), "head_dim 80 has no attention instantiation"),
    (dict(dim=304, n_heads=1, n_kv_heads=1), "dim % 32 == 0"),
    (dict(vocab_size=32001), "vocab_size 32001 must be a multiple of 4"),
    (dict(n_heads=6, n_kv_heads=4), "n_heads % n_kv_heads"),
])
def test_create_rejects_unsupported_shapes_before_touching_a_device(kw, msg):
    """Shape limits of the kernels are checked up front with a message (no GPU needed)."""
    d = dict(dim=288, n_layers=6, n_heads=6, n_kv_heads=6, vocab_size=32000, hidden_dim=768,
             max_seq_len=256, max_batch_size=1, norm_eps=1e-6)
    d.update(kw)
    with pytest.raises(RuntimeError, match=re.escape(msg)):
        l3hip.Context(l3hip.Dims(**d), 0)
