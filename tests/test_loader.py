"""Streaming .npz reader (utils.StreamingNpz) against the reference's
loader: ``utils.load_parameters`` is ``np.load`` (reference utils.py:4-5), so every member
read by the fast path must equal ``np.load``'s array bit for bit, whatever the member's
layout, and members the fast path does not take must come back through ``np.load``."""

import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "llama3.np_amd"))
import utils  # noqa: E402


def _members(rng):
    return {
        "model.embed_tokens.weight": rng.standard_normal((97, 64), dtype=np.float32),
        "model.norm.weight": rng.standard_normal(64, dtype=np.float32),
        "scalar": np.float32(3.5),
        "empty": np.zeros((0, 8), np.float32),
        "f64": rng.standard_normal((5, 3)),                       # another dtype: fallback
        "fortran": np.asfortranarray(rng.standard_normal((6, 4), dtype=np.float32)),
        "big_endian": rng.standard_normal(7).astype(">f4"),      # not <f4: fallback
    }


@pytest.mark.parametrize("compressed", [False, True])
def test_streaming_npz_equals_np_load(tmp_path, compressed):
    path = str(tmp_path / "w.npz")
    m = _members(np.random.default_rng(0))
    (np.savez_compressed if compressed else np.savez)(path, **m)
    ref = np.load(path, allow_pickle=False)
    made = []

    def alloc(shape, dtype):
        a = np.empty(shape, dtype)
        made.append(a)
        return a

    s = utils.StreamingNpz(path, alloc)
    assert set(s.keys()) == set(ref.files)
    for k in ref.files:
        got, want = s.get(k), ref[k]
        assert got.dtype == want.dtype and got.shape == want.shape, k
        np.testing.assert_array_equal(got, want, err_msg=k)
    assert s.get("missing") is None and s.get("missing", 7) == 7
    assert "model.norm.weight" in s
    with pytest.raises(KeyError):
        s["missing"]
    # stored members of the fast-path layout land in the caller's buffers; compressed ones never
    assert len(made) == (0 if compressed else 4)
    s.close()


def test_streaming_npz_detects_truncation(tmp_path):
    path = str(tmp_path / "w.npz")
    np.savez(path, a=np.arange(4096, dtype=np.float32))
    with open(path, "rb") as f:
        blob = f.read()
    cut = str(tmp_path / "cut.npz")
    # keep the central directory (so the zip opens) but lose data bytes of the member
    import zipfile

    zi = zipfile.ZipFile(path).getinfo("a.npy")
    data_end = zi.header_offset + 30 + len(zi.filename) + len(zi.extra) + zi.file_size
    with open(cut, "wb") as f:
        f.write(blob[: data_end - 1000] + blob[data_end:])
    s = utils.StreamingNpz(cut, lambda shape, dtype: np.empty(shape, dtype))
    with pytest.raises((ValueError, OSError)):
        s.get("a")


def test_streaming_npz_threaded_pieces(tmp_path):
    """A member larger than one read piece is copied by several threads; every byte lands."""
    path = str(tmp_path / "w.npz")
    a = np.random.default_rng(3).standard_normal((301, 257), dtype=np.float32)
    np.savez(path, a=a, b=a[:7])
    s = utils.StreamingNpz(path, lambda shape, dtype: np.empty(shape, dtype), threads=4)
    s.CHUNK = 4096 + 12  # pieces not aligned to rows or pages
    np.testing.assert_array_equal(s.get("a"), a)
    np.testing.assert_array_equal(s["b"], a[:7])
    s.close()


def test_recycling_alloc_reuses_dropped_blocks():
    """A member's buffer returns to the free list once the array and its views are gone."""
    pool = utils.RecyclingAlloc(keep=2)
    a = pool((4, 8), np.float32)
    a[:] = 1
    t = a.T  # a view keeps the block alive
    addr = a.__array_interface__["data"][0]
    del a
    b = pool((4, 8), np.float32)
    assert b.__array_interface__["data"][0] != addr
    del t
    c = pool((8, 4), np.float32)  # same byte size: the freed block comes back
    assert c.__array_interface__["data"][0] == addr
    pool.clear()
    del b, c
    assert not pool._free


def test_llama_refuses_missing_weights_before_any_device_call():
    """Llama.__init__ checks every tensor the forward reads (utils.weight_names) before it
    creates a device context: a mapping without one raises KeyError here, on a CPU-only host
    (the reference fails late, AttributeError on None.T, llama3.py:133-136)."""
    import llama3
    import synth
    from utils import weight_names

    args = synth.tiny(1)
    w = synth.make_weights(args, synth.TINY_HIDDEN, seed=1)
    assert sorted(weight_names(args.n_layers)) == sorted(w)
    del w["model.layers.1.mlp.up_proj.weight"]
    with pytest.raises(KeyError, match="up_proj"):
        llama3.Llama(w, args)
