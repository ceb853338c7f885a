"""Synthetic weight sets with the reference's tensor names and shapes.

The real ``stories15M.model.npz`` is absent (reference ``.MISSING_LARGE_BLOBS:1``)
and there is no network, so every test and benchmark runs on weights drawn
here from a fixed seed.  Keys and layouts follow
``llama3.py:219-237,269,280-281``: projections are ``[out, in]`` row-major
fp32, norms are ``[dim]``.

Two presets:

* ``"default"`` — projections N(0, 0.02^2), embedding N(0, 1), norms = 1.
* ``"sharp"``   — projections N(0, 0.08^2) and lm_head scaled x6 so logits
  reach |36| and greedy decoding has clear top-1 margins (parity of greedy
  ids needs margins far above the fp32-vs-fp64 logit error).

Generation is deterministic for a given NumPy build (PCG64 + ziggurat), and
``digest()`` gives a sha256 over the arrays so fixtures can assert they were
made from the same weights.
"""

import hashlib
from typing import Dict, Optional

import numpy as np

from config import ModelArgs

PRESETS = {
    "default": dict(std=0.02, emb_std=1.0, lm_scale=1.0),
    "sharp": dict(std=0.08, emb_std=1.0, lm_scale=6.0),
}


def make_weights(args: ModelArgs, hidden_dim: int, seed: int = 0,
                 preset: str = "default") -> Dict[str, np.ndarray]:
    cfg = PRESETS[preset]
    rng = np.random.default_rng(seed)
    D, H, KVH = args.dim, args.n_heads, args.kv_heads
    HD = D // H

    def normal(shape, std):
        return (rng.standard_normal(shape, dtype=np.float32) * np.float32(std)).astype(np.float32)

    w = {"model.embed_tokens.weight": normal((args.vocab_size, D), cfg["emb_std"])}
    for i in range(args.n_layers):
        p = f"model.layers.{i}."
        w[p + "self_attn.q_proj.weight"] = normal((H * HD, D), cfg["std"])
        w[p + "self_attn.k_proj.weight"] = normal((KVH * HD, D), cfg["std"])
        w[p + "self_attn.v_proj.weight"] = normal((KVH * HD, D), cfg["std"])
        w[p + "self_attn.o_proj.weight"] = normal((D, H * HD), cfg["std"])
        w[p + "mlp.gate_proj.weight"] = normal((hidden_dim, D), cfg["std"])
        w[p + "mlp.up_proj.weight"] = normal((hidden_dim, D), cfg["std"])
        w[p + "mlp.down_proj.weight"] = normal((D, hidden_dim), cfg["std"])
        w[p + "input_layernorm.weight"] = np.ones(D, np.float32)
        w[p + "post_attention_layernorm.weight"] = np.ones(D, np.float32)
    w["model.norm.weight"] = np.ones(D, np.float32)
    w["lm_head.weight"] = normal((args.vocab_size, D), cfg["std"] * cfg["lm_scale"])
    return w


def pool_weights(args: ModelArgs, hidden_dim: int, seed: int = 0, pool_floats: int = 1 << 28,
                 std: float = 0.02, emb_scale: float = 50.0,
                 rng: Optional[np.random.Generator] = None) -> Dict[str, np.ndarray]:
    """Weights for shapes too large to draw tensor by tensor (the 32-layer Llama-3-8B shape is
    8.5G floats): one uniform pool of ``pool_floats`` values with standard deviation ``std``,
    every projection a contiguous view of it at a random offset (no copy), the embedding the
    pool scaled by ``emb_scale`` and tiled to [VS, D] (std ~1 at the default), norms = 1.  Same
    keys and [out, in] layouts as ``make_weights``; the draw order is fixed, so a seed gives the
    same weights here and in bench.py's Llama-3-shape runs (which pass their own ``rng`` and
    draw their token ids from it afterwards)."""
    rng = np.random.default_rng(seed) if rng is None else rng
    pool = (rng.random(pool_floats, dtype=np.float32) * 2 - 1) * np.float32(std * 3 ** 0.5)
    D, H, KVH, VS = args.dim, args.n_heads, args.kv_heads, args.vocab_size
    HD = D // H

    def view(shape):
        n = int(np.prod(shape))
        if n <= pool.size:
            o = int(rng.integers(0, pool.size - n + 1))
            return pool[o:o + n].reshape(shape)
        return np.resize(pool, n).reshape(shape)

    w = {"model.embed_tokens.weight": np.resize(pool * np.float32(emb_scale), VS * D).reshape(VS, D)}
    for i in range(args.n_layers):
        p = f"model.layers.{i}."
        w[p + "self_attn.q_proj.weight"] = view((H * HD, D))
        w[p + "self_attn.k_proj.weight"] = view((KVH * HD, D))
        w[p + "self_attn.v_proj.weight"] = view((KVH * HD, D))
        w[p + "self_attn.o_proj.weight"] = view((D, H * HD))
        w[p + "mlp.gate_proj.weight"] = view((hidden_dim, D))
        w[p + "mlp.up_proj.weight"] = view((hidden_dim, D))
        w[p + "mlp.down_proj.weight"] = view((D, hidden_dim))
        w[p + "input_layernorm.weight"] = np.ones(D, np.float32)
        w[p + "post_attention_layernorm.weight"] = np.ones(D, np.float32)
    w["model.norm.weight"] = np.ones(D, np.float32)
    w["lm_head.weight"] = view((VS, D))
    return w


def digest(weights: Dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(weights):
        h.update(k.encode())
        h.update(np.ascontiguousarray(weights[k]).tobytes())
    return h.hexdigest()


def save_npz(path: str, weights: Dict[str, np.ndarray]) -> None:
    np.savez(path, **weights)


def stories15m(max_batch_size: int = 1) -> ModelArgs:
    """stories15M shape (reference config.py defaults); FD = 768."""
    return ModelArgs(max_batch_size=max_batch_size)


STORIES15M_HIDDEN = 768


def tiny(max_batch_size: int = 4) -> ModelArgs:
    """Small model for committed golden fixtures."""
    return ModelArgs(dim=64, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=512,
                     max_seq_len=64, max_batch_size=max_batch_size)


TINY_HIDDEN = 192


def llama3_shape(n_layers: int = 32, max_batch_size: int = 64, max_seq_len: int = 2048) -> ModelArgs:
    """Llama-3-8B-shaped config (BASELINE.json configs[4]); FD = 14336."""
    return ModelArgs(dim=4096, n_layers=n_layers, n_heads=32, n_kv_heads=8,
                     vocab_size=128256, max_seq_len=max_seq_len, max_batch_size=max_batch_size)


LLAMA3_HIDDEN = 14336
