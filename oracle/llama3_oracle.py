"""ORACLE — test infrastructure only.  CPU restatement of the reference forward.

This module restates, in plain NumPy, exactly the arithmetic of the reference
``llama3.py`` (swap357/llama3.np @ 2025-05-23) so that the MI355X path can be
checked against it on the GPU box, where ``/root/reference`` does not exist.

RULES (see DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this module, and only as the checker /
    the reported CPU baseline.  The product package (``llama3.np_amd/``)
    never imports it; its forward fails loudly without the HIP library.
  * The restatement must reproduce the reference's dtype flow bit-for-bit:
    fp32 embedding and layer-0 RMSNorm + QKV; f64 RoPE tables
    (``llama3.py:31-38``) promote q/k to f64; f64 KV caches
    (``llama3.py:138-153``) promote everything after RoPE, and every later
    layer, to f64; logits are f64 ``[B, 1, VS]`` (``llama3.py:307``).
  * It keeps the same NumPy op sequence (same views, same broadcasting) so
    OpenBLAS takes the same code paths — pinned against fixtures produced by
    importing the reference itself (``tests/golden/make_golden.py``) at
    max-abs <= 1e-12 (``tests/test_oracle_golden.py``).

Parity pinned: yes — by the reference's own outputs on synthetic weights
(committed fixtures), because the reference ships no golden vectors.
"""

import math
from typing import Iterator, Mapping, Optional

import numpy as np

NEG_INF = float("-inf")


# ---- element ops -----------------------------------------------------------

def softmax(x):
    """llama3.py:22-24 — subtract row max, exp, divide by row sum."""
    e = np.exp(x - np.max(x, axis=-1, keepdims=True))
    return e / np.sum(e, axis=-1, keepdims=True)


def silu(x):
    """llama3.py:27-28 — x * (1 / (1 + exp(-x)))."""
    return x * (1 / (1 + np.exp(-x)))


def rope_tables(head_dim: int, max_seq_len: int, base: int = 10000):
    """llama3.py:31-38 — f64 cos/sin of pos * base^(-2i/HD); base fixed at 1e4."""
    exponents = np.arange(0, head_dim, 2)[: head_dim // 2] / head_dim
    inv_freq = 1.0 / (base ** exponents)
    angles = np.outer(np.arange(max_seq_len), inv_freq)
    return np.cos(angles), np.sin(angles)


def rope(xq, xk, cos, sin):
    """llama3.py:41-76 — interleaved-pair rotation (x[2i], x[2i+1])."""
    c = np.expand_dims(cos, axis=(0, 2))
    s = np.expand_dims(sin, axis=(0, 2))

    def rotate(x):
        pairs = x.reshape(x.shape[:-1] + (-1, 2))
        re, im = np.split(pairs, 2, axis=-1)
        re = re.squeeze(-1)
        im = im.squeeze(-1)
        out = np.stack([re * c - im * s, re * s + im * c], axis=-1)
        return out.reshape(out.shape[:-2] + (-1,))

    return rotate(xq), rotate(xk)


def repeat_kv(x, n_rep: int):
    """llama3.py:79-83 — each KV head repeated n_rep times, contiguously."""
    return x if n_rep == 1 else np.repeat(x, n_rep, axis=2)


def rmsnorm(x, weight, eps):
    """llama3.py:111-114 — (x / sqrt(mean(x^2) + eps)) * w, in x's dtype."""
    ms = (x ** 2).mean(-1, keepdims=True) + eps
    return (x / np.sqrt(ms)) * weight


def ffn(x, w_gate, w_up, w_down):
    """llama3.py:97-103 with W stored [out, in]; weights are used through .T views."""
    g = silu(x @ w_gate.T)
    u = x @ w_up.T
    return (g * u) @ w_down.T


def causal_mask(L: int, start_pos: int):
    """llama3.py:293-297 — -inf strictly above the diagonal, zero prefix of width start_pos."""
    if L <= 1:
        return None
    m = np.triu(np.full((L, L), NEG_INF), k=1)
    return np.concatenate([np.zeros((L, start_pos)), m], axis=1)


# ---- model -----------------------------------------------------------------

class OracleLayer:
    """One transformer block with its persistent f64 KV cache (llama3.py:117-261)."""

    def __init__(self, w: Mapping[str, np.ndarray], i: int, args):
        p = f"model.layers.{i}."
        self.wq = w[p + "self_attn.q_proj.weight"]
        self.wk = w[p + "self_attn.k_proj.weight"]
        self.wv = w[p + "self_attn.v_proj.weight"]
        self.wo = w[p + "self_attn.o_proj.weight"]
        self.wg = w[p + "mlp.gate_proj.weight"]
        self.wu = w[p + "mlp.up_proj.weight"]
        self.wd = w[p + "mlp.down_proj.weight"]
        self.n_attn = w[p + "input_layernorm.weight"]
        self.n_ffn = w[p + "post_attention_layernorm.weight"]
        self.eps = args.norm_eps
        self.H = args.n_heads
        self.KVH = args.n_heads if args.n_kv_heads is None else args.n_kv_heads
        self.HD = args.dim // args.n_heads
        shape = (args.max_batch_size, args.max_seq_len, self.KVH, self.HD)
        self.cache_k = np.zeros(shape)  # f64, as llama3.py:138-153
        self.cache_v = np.zeros(shape)

    def attention(self, x, start_pos, mask, cos, sin):
        B, L, _ = x.shape
        q = (x @ self.wq.T).reshape(B, L, self.H, self.HD)
        k = (x @ self.wk.T).reshape(B, L, self.KVH, self.HD)
        v = (x @ self.wv.T).reshape(B, L, self.KVH, self.HD)
        q, k = rope(q, k, cos, sin)
        end = start_pos + L
        self.cache_k[:B, start_pos:end] = k
        self.cache_v[:B, start_pos:end] = v
        n_rep = self.H // self.KVH
        keys = repeat_kv(self.cache_k[:B, :end], n_rep).transpose(0, 2, 1, 3)
        vals = repeat_kv(self.cache_v[:B, :end], n_rep).transpose(0, 2, 1, 3)
        q = q.transpose(0, 2, 1, 3)
        scores = q @ keys.transpose(0, 1, 3, 2) / math.sqrt(self.HD)
        if mask is not None:
            scores = scores + mask[None, None, :, :]
        o = softmax(scores) @ vals
        o = o.transpose(0, 2, 1, 3).reshape(B, L, -1)
        return o @ self.wo.T

    def __call__(self, x, start_pos, mask, cos, sin):
        z = x + self.attention(rmsnorm(x, self.n_attn, self.eps), start_pos, mask, cos, sin)
        return z + ffn(rmsnorm(z, self.n_ffn, self.eps), self.wg, self.wu, self.wd)


class OracleModel:
    """Whole forward + greedy loop (llama3.py:264-321), caches persistent across calls."""

    def __init__(self, weights: Mapping[str, np.ndarray], args):
        self.args = args
        self.emb = weights["model.embed_tokens.weight"]
        self.cos, self.sin = rope_tables(args.dim // args.n_heads, args.max_seq_len)
        self.layers = [OracleLayer(weights, i, args) for i in range(args.n_layers)]
        self.final_norm = weights["model.norm.weight"]
        self.lm_head = weights["lm_head.weight"]

    def __call__(self, input_ids, start_pos: int):
        L = input_ids.shape[1]
        h = self.emb[input_ids]
        cos = self.cos[start_pos:start_pos + L]
        sin = self.sin[start_pos:start_pos + L]
        mask = causal_mask(L, start_pos)
        for layer in self.layers:
            h = layer(h, start_pos, mask, cos, sin)
        h = rmsnorm(h, self.final_norm, self.args.norm_eps)
        return h[:, [-1], :] @ self.lm_head.T

    def generate(self, input_ids, max_new_tokens: int) -> Iterator[np.ndarray]:
        """llama3.py:310-321, including the position quirk: decode step i>=1
        runs at pos = L + i, so cache slot L is never written (stays zero)."""
        L = input_ids.shape[1]
        nxt: Optional[np.ndarray] = None
        for i, pos in enumerate(range(L, max_new_tokens)):
            if i == 0:
                logits = self(input_ids, 0)
            else:
                logits = self(nxt, pos)
            nxt = logits[:, -1, :].argmax(-1, keepdims=True)
            yield nxt


def greedy_ids(model: OracleModel, input_ids, max_new_tokens: int):
    """All ids the reference loop yields, as int64 [B, steps]."""
    return np.concatenate(list(model.generate(input_ids, max_new_tokens)), axis=1)
