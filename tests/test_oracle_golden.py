"""Pin the oracle to the reference's own outputs (CPU, no GPU).

The fixtures were produced by importing the reference (tests/golden/make_golden.py).
The oracle restates the same NumPy op sequence, so agreement is expected at
float64 round-off (<= 1e-12), far tighter than the 1e-4 GPU parity bar.
"""

import os

import numpy as np
import pytest

import llama3_oracle as orc
import synth
from conftest import load_golden

TIGHT = 1e-12


def test_ops_known_answers():
    g = load_golden("ops")
    np.testing.assert_array_equal(orc.softmax(g["softmax_x"]), g["softmax_y"])
    np.testing.assert_array_equal(orc.softmax(g["softmax_masked_x"]), g["softmax_masked_y"])
    np.testing.assert_array_equal(orc.silu(g["silu_x"]), g["silu_y"])
    c, s = orc.rope_tables(48, 256)
    np.testing.assert_array_equal(c, g["rope_cos"])
    np.testing.assert_array_equal(s, g["rope_sin"])
    st = int(g["rope_start"])
    q, k = orc.rope(g["rope_xq"], g["rope_xk"], c[st:st + 8], s[st:st + 8])
    np.testing.assert_array_equal(q, g["rope_q"])
    np.testing.assert_array_equal(k, g["rope_k"])
    np.testing.assert_array_equal(orc.rmsnorm(g["rms_x"], g["rms_w"], 1e-6), g["rms_y"])
    np.testing.assert_array_equal(orc.rmsnorm(g["rms64_x"], g["rms_w"], 1e-6), g["rms64_y"])
    y = orc.ffn(g["ffn_x"], g["ffn_wg"], g["ffn_wu"], g["ffn_wd"])
    np.testing.assert_allclose(y, g["ffn_y"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(orc.repeat_kv(g["repkv_x"], 3), g["repkv_y"])


def _weights_for(g, args, hidden):
    w = synth.make_weights(args, hidden, seed=int(g["seed"]), preset=str(g["preset"]))
    assert synth.digest(w) == str(g["weights_sha256"]), "synthetic weight generator drifted"
    return w


@pytest.mark.parametrize("name", ["tiny", "stories15m_default", "stories15m_sharp"])
def test_oracle_forward_matches_reference(name):
    g = load_golden(name)
    if name == "tiny":
        args, hidden, tags = synth.tiny(4), synth.TINY_HIDDEN, ["prefill", "chunk", "decode"]
    else:
        args, hidden, tags = synth.stories15m(2), synth.STORIES15M_HIDDEN, ["prefill"]
    m = orc.OracleModel(_weights_for(g, args, hidden), args)
    for t in tags:  # sequential on one model: persistent caches, like the reference
        out = m(g[f"{t}_ids"], int(g[f"{t}_start"]))
        assert out.dtype == np.float64 and out.shape == g[f"{t}_logits"].shape
        assert np.max(np.abs(out - g[f"{t}_logits"])) <= TIGHT


def test_oracle_greedy_tiny_matches_reference():
    g = load_golden("tiny")
    args = synth.tiny(4)
    m = orc.OracleModel(_weights_for(g, args, synth.TINY_HIDDEN), args)
    ids = orc.greedy_ids(m, g["gen_prompt"], int(g["gen_max_new"]))
    np.testing.assert_array_equal(ids, g["gen_ids"])
    zero = np.nonzero(np.all(m.layers[0].cache_k[0] == 0, axis=(1, 2)))[0][:8]
    np.testing.assert_array_equal(zero, g["gen_zero_slots"])  # the decode hole


@pytest.mark.slow
@pytest.mark.parametrize("name", ["stories15m_default", "stories15m_sharp"])
def test_oracle_greedy_stories_matches_reference(name):
    g = load_golden(name)
    args = synth.stories15m(2)
    m = orc.OracleModel(_weights_for(g, args, synth.STORIES15M_HIDDEN), args)
    ids = orc.greedy_ids(m, g["dream_prompt"], int(g["dream_max_new"]))
    np.testing.assert_array_equal(ids, g["dream_ids"])
    assert int(g["dream_zero_slots"][0]) == g["dream_prompt"].shape[1]  # slot L never written


@pytest.mark.skipif(not os.environ.get("L3_SLOW_TESTS"),
                    reason="Llama-3-shape slice: 6 GB of weights, ~1.5 min (set L3_SLOW_TESTS=1)")
def test_oracle_c5_slice_matches_reference():
    """2-layer Llama-3-8B shape (GQA n_rep 4, HD 128), B = 1, L = 256
    prefill then decode at positions 257 and 258 (slot 256 is the decode hole)."""
    g = load_golden("c5_slice")
    args = synth.llama3_shape(n_layers=2, max_batch_size=1)
    m = orc.OracleModel(_weights_for(g, args, synth.LLAMA3_HIDDEN), args)
    for t in ["prefill", "dec1", "dec2"]:
        out = m(g[f"{t}_ids"], int(g[f"{t}_start"]))
        assert np.max(np.abs(out - g[f"{t}_logits"])) <= TIGHT
