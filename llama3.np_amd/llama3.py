"""MI355X drop-in for the reference's ``llama3.py`` (swap357/llama3.np).

Same public surface — ``Llama``, ``TransformerBlock``, ``Attention``,
``FeedForward``, ``RMSNorm``, ``softmax``, ``silu``, ``compute_cos_sin_cache``,
``apply_rotary_emb``, ``repeat_kv`` and the ``__main__`` CLI — with the
arithmetic executed by hand-written gfx950 HIP kernels through the C ABI in
``include/llama3hip.h`` (``l3hip.py``).  There is no NumPy fallback: without
``libllama3hip.so`` or without a HIP device every compute call raises.

Differences from the reference, all deliberate:

* arithmetic is fp32 everywhere (the reference promotes to f64 after RoPE,
  ``llama3.py:181``, via its f64 tables and caches); logits are returned as
  float32 ``[B, 1, VS]``.  Parity is to tolerance.
* ``TransformerBlock.__call__`` / ``Attention.__call__`` accept ``mask`` and
  ``freqs_cos/freqs_sin`` for signature compatibility but rebuild the causal
  mask and RoPE angles on the device from ``(start_pos, L)`` — the reference's
  callers always pass exactly those (``llama3.py:289-297``); shapes are checked.
* ``compute_cos_sin_cache`` stays a host function (init-time f64 tables, as
  ``llama3.py:31-38``); the device builds its own fp32 copy of the same table.
* the module functions ``softmax``, ``silu``, ``apply_rotary_emb``, ``repeat_kv``
  and ``RMSNorm.__call__`` are host NumPy with the reference's exact semantics
  (dtype kept, results bit-identical): the forward never calls them — its
  versions are fused into the kernels — and the reference's own tests check
  them with ``==``.

Everything the reference keeps on the object (``args``, ``tok_embedding``,
``freqs_cos/sin``, ``layers``, ``norm``, ``lm_head_weight``, per-class weight
views) is kept, so introspecting code keeps working.
"""

from __future__ import annotations

import os
import sys
import time
import zipfile
from typing import Iterator, Mapping, Optional, Sequence

import numpy as np

import l3hip
from config import ModelArgs
from tokenizer import Tokenizer
from utils import RecyclingAlloc, StreamingNpz, load_parameters, weight_names

# .npz reader (A/B: tools/load_probe.py): "threads" — utils.StreamingNpz into ordinary arrays,
# recycled when host copies are not kept (default), "pinned" — into recycled page-locked buffers
# when host copies are not kept, "npzfile" — NumPy's NpzFile as the reference's load_parameters
_NPZ_READER = os.environ.get("L3_NPZ_READER", "threads")

DEFAULT_DEVICE = int(os.environ.get("LLAMA3_HIP_DEVICE", "0"))


# ---- module functions (reference llama3.py:22-83) ----------------------------
#
# Host NumPy, as in the reference, so the module API keeps its exact semantics: the input
# dtype is kept (an f64 masked-score array stays f64) and the results are bit-identical to the
# reference's (its own suite compares them with ==, tests/test_llama_implementations.py:55-111;
# here tests/test_module_api.py against the reference-generated tests/golden/ops.npz).  The
# device forward never calls them: there the same arithmetic is fused into the HIP kernels
# (softmax and mask in attn_fwd_kernel, RoPE in the QKV GEMM epilogue, RMSNorm as a row factor
# of the consuming GEMM); the standalone GPU op kernels stay reachable as l3hip.Context.op_*.

def softmax(x):
    """Row softmax over the last axis, input dtype kept (reference llama3.py:22-24)."""
    e = np.exp(x - np.max(x, axis=-1, keepdims=True))
    return e / np.sum(e, axis=-1, keepdims=True)


def silu(x):
    """x * (1 / (1 + exp(-x))), input dtype kept (reference llama3.py:27-28)."""
    return x * (1 / (1 + np.exp(-x)))


def compute_cos_sin_cache(head_dim: int, max_seq_len: int, base: int = 10000):
    """Host f64 RoPE tables, same formula as reference llama3.py:31-38."""
    inv_freq = 1.0 / (base ** (np.arange(0, head_dim, 2)[: head_dim // 2] / head_dim))
    ang = np.outer(np.arange(max_seq_len), inv_freq)
    return np.cos(ang), np.sin(ang)


def _rotate_pairs(x, c, s):
    """(x[2i], x[2i+1]) rotated by the angle whose cos / sin are c / s (broadcast [1,L,1,HD/2])."""
    pairs = x.reshape(x.shape[:-1] + (-1, 2))
    re, im = pairs[..., 0], pairs[..., 1]
    out = np.stack([re * c - im * s, re * s + im * c], axis=-1)
    return out.reshape(out.shape[:-2] + (-1,))


def apply_rotary_emb(xq, xk, freqs_cos, freqs_sin):
    """Interleaved-pair RoPE of q and k (reference llama3.py:41-76); the result takes the
    promoted dtype of the inputs and tables (f64 with the reference's f64 tables)."""
    c = np.expand_dims(freqs_cos, axis=(0, 2))
    s = np.expand_dims(freqs_sin, axis=(0, 2))
    return _rotate_pairs(xq, c, s), _rotate_pairs(xk, c, s)


def repeat_kv(x, n_rep: int):
    """GQA head expansion (reference llama3.py:79-83).

    Pure data movement; inside the device forward the expansion is an index
    map (query head h reads KV head h // n_rep), never a copy."""
    if n_rep == 1:
        return x
    return np.repeat(x, n_rep, axis=2)


# ---- layers ------------------------------------------------------------------

def _dims(args: ModelArgs, hidden_dim: int, n_layers: int, vocab_size: int) -> l3hip.Dims:
    kvh = args.n_heads if args.n_kv_heads is None else args.n_kv_heads
    return l3hip.Dims(dim=args.dim, n_layers=n_layers, n_heads=args.n_heads, n_kv_heads=kvh,
                      vocab_size=vocab_size, hidden_dim=hidden_dim, max_seq_len=args.max_seq_len,
                      max_batch_size=args.max_batch_size, norm_eps=args.norm_eps)


def _check_freqs(freqs_cos, freqs_sin, L: int, head_dim: int) -> None:
    for f in (freqs_cos, freqs_sin):
        if f is not None and np.shape(f) != (L, head_dim // 2):
            raise ValueError(f"freqs shape {np.shape(f)} does not match (L={L}, HD/2={head_dim // 2})")


class _Dropped:
    """Placeholder for a host weight not kept by a streaming load (keep_host_weights=False):
    the tensor lives only in HBM; host-side uses of it raise."""

    def __init__(self, shape):
        self.shape = tuple(shape)

    @property
    def T(self):
        return _Dropped(self.shape[::-1])

    def __array__(self, *a, **k):
        raise RuntimeError("host copy not kept (Llama(..., keep_host_weights=False))")


class FeedForward:
    """SwiGLU MLP (reference llama3.py:86-103): one fused gate|up MFMA GEMM with a
    silu(g)*u epilogue, then the down GEMM, on the GPU.

    Unlike the module functions above this stays a device call: it is the metric's kernel
    pair, and a standalone call is how a user reaches it outside a whole
    forward.  The arithmetic is fp32 (as the forward); the result is returned in the dtype
    the reference's ``x @ W`` would produce (``np.result_type(x, W)``), so the reference's
    dtype contract holds, but the values match it to fp32 tolerance, not bit for bit (the
    reference's own suite pins FeedForward only through the full forward at 1e-4,
    tests/test_llama_implementations.py:114-179)."""

    def __init__(self, up_weight, gate_weight, down_weight):
        self.up_weight = up_weight.T
        self.gate_weight = gate_weight.T
        self.down_weight = down_weight.T

    def __call__(self, x):
        x = np.asarray(x)
        ctx = l3hip.op_context(DEFAULT_DEVICE)
        y = ctx.op_ffn(x.reshape(-1, x.shape[-1]), self.gate_weight.T, self.up_weight.T,
                       self.down_weight.T)
        out_t = np.result_type(x.dtype, self.gate_weight.dtype, self.down_weight.dtype)
        return y.reshape(x.shape).astype(out_t, copy=False)


class RMSNorm:
    """x / sqrt(mean(x^2) + eps) * w on the host, input dtype kept (reference
    llama3.py:106-114; bit-identical to it, see the module functions' note).  Inside the
    device forward the norm is a row factor of the consuming GEMM."""

    def __init__(self, weight, eps: float):
        self.weight = weight
        self.eps = eps

    def __call__(self, x):
        z = (x ** 2).mean(-1, keepdims=True) + self.eps
        return (x / np.sqrt(z)) * self.weight


class Attention:
    """Causal GQA attention with a persistent device KV cache (reference llama3.py:117-213).

    Owned by a ``TransformerBlock`` it shares that block's device state
    (cache included), exactly as the reference's Attention owns the cache the
    block uses.  Constructed alone it gets a private one-layer context."""

    def __init__(self, q_weight, k_weight, v_weight, o_weight, args: ModelArgs,
                 _bind: Optional[tuple] = None):
        self.n_kv_heads = args.n_heads if args.n_kv_heads is None else args.n_kv_heads
        assert args.n_heads % self.n_kv_heads == 0
        self.n_local_heads = args.n_heads
        self.n_local_kv_heads = self.n_kv_heads
        self.n_rep = self.n_local_heads // self.n_local_kv_heads
        self.head_dim = args.dim // args.n_heads
        self.q_weight = q_weight.T
        self.k_weight = k_weight.T
        self.v_weight = v_weight.T
        self.o_weight = o_weight.T
        if _bind is None:
            ctx = l3hip.Context(_dims(args, 32, 1, 0), DEFAULT_DEVICE)
            for kind, w in ((l3hip.W_Q, q_weight), (l3hip.W_K, k_weight), (l3hip.W_V, v_weight),
                            (l3hip.W_O, o_weight)):
                ctx.upload(0, kind, w)
            ctx.finalize()
            _bind = (ctx, 0)
        self._ctx, self._layer = _bind

    def __call__(self, x, start_pos: int, mask, freqs_cos, freqs_sin):
        x = np.asarray(x)
        _check_freqs(freqs_cos, freqs_sin, x.shape[1], self.head_dim)
        return self._ctx.attention_forward(self._layer, x, start_pos)


class TransformerBlock:
    """Pre-norm block (reference llama3.py:216-261) executed as 4 MFMA GEMMs with
    fused epilogues plus one fused attention kernel (kernel list)."""

    def __init__(self, weight: dict, layer_id: int, args: ModelArgs, _bind: Optional[tuple] = None,
                 _keep_host: bool = True):
        p = f"model.layers.{layer_id}."
        names = {
            l3hip.W_Q: p + "self_attn.q_proj.weight", l3hip.W_K: p + "self_attn.k_proj.weight",
            l3hip.W_V: p + "self_attn.v_proj.weight", l3hip.W_O: p + "self_attn.o_proj.weight",
            l3hip.W_GATE: p + "mlp.gate_proj.weight", l3hip.W_UP: p + "mlp.up_proj.weight",
            l3hip.W_DOWN: p + "mlp.down_proj.weight",
            l3hip.W_ATTN_NORM: p + "input_layernorm.weight",
            l3hip.W_FFN_NORM: p + "post_attention_layernorm.weight",
        }
        w = {}
        for kind, name in names.items():
            t = weight.get(name)
            if t is None:  # the reference fails later with AttributeError on None.T
                raise KeyError(f"missing weight {name!r}")
            w[kind] = t
        if _bind is None:
            ctx = l3hip.Context(_dims(args, w[l3hip.W_GATE].shape[0], 1, 0), DEFAULT_DEVICE)
            _bind = (ctx, 0)
            standalone = True
        else:
            standalone = False
        self._ctx, self._layer = _bind
        for kind, t in w.items():
            self._ctx.upload(self._layer, kind, t)
        if standalone:
            self._ctx.finalize()
        if not _keep_host:  # streaming load: the device copy is the only copy
            w = {k: _Dropped(v.shape) for k, v in w.items()}
        self.attention = Attention(w[l3hip.W_Q], w[l3hip.W_K], w[l3hip.W_V], w[l3hip.W_O], args,
                                   _bind=_bind)
        self.feed_forward = FeedForward(w[l3hip.W_UP], w[l3hip.W_GATE], w[l3hip.W_DOWN])
        self.input_layernorm = RMSNorm(w[l3hip.W_ATTN_NORM], eps=args.norm_eps)
        self.post_attention_layernorm = RMSNorm(w[l3hip.W_FFN_NORM], eps=args.norm_eps)
        self._head_dim = args.dim // args.n_heads

    def __call__(self, x, start_pos: int, mask, freqs_cos, freqs_sin):
        x = np.asarray(x)
        _check_freqs(freqs_cos, freqs_sin, x.shape[1], self._head_dim)
        return self._ctx.layer_forward(self._layer, x, start_pos)


class Llama:
    """The whole forward + greedy loop (reference llama3.py:264-321).

    Weights are uploaded once to HBM; ``__call__`` keeps activations
    device-resident across all layers and copies back only the last-position
    logits (the last block runs its attention / O-proj / FFN for that position only
    — the only rows llama3.py:304 keeps — while its K / V cache append still covers
    every position; ``context.set_last_layer_rows(True)`` runs every row).
    ``generate`` runs argmax on the device and copies back only ids."""

    def __init__(self, model_path: str, args: ModelArgs, device: Optional[int] = None,
                 keep_host_weights: bool = True, devices: Optional[Sequence[int]] = None):
        """``device`` / ``keep_host_weights`` / ``devices`` are extensions.

        ``devices=[0, ..., N-1]``: one process drives N GPUs (``l3hip.Group``, the C ABI's
        l3_group_*).  Every call keeps the reference's signature and result: batch row r runs on
        ``devices[r % N]`` (rows never interact, llama3.py:163-211), the other devices' logits
        rows reach the first device in one RCCL gather over xGMI, and ``__call__`` returns the
        full ``[B, 1, VS]``; a single prompt (B = 1) runs on the first device alone, greedy
        decode included.  Only the constructor changes for a reference user.  With
        ``keep_host_weights=False`` every ``.npz`` member is read, uploaded to HBM and
        dropped before the next is read (NumPy's NpzFile reads members lazily), so host
        memory peaks at one tensor instead of the whole checkpoint (32 GB for the
        Llama-3-8B shape); the reference-style host attributes then hold placeholders.
        ``model_path`` may also be a mapping of the ``.npz`` keys to arrays (what
        ``load_parameters`` returns; extension) — uploaded as given, no file read."""
        self.args = args
        keep = keep_host_weights
        pool = None
        if isinstance(model_path, Mapping):
            weight = model_path
        elif _NPZ_READER == "npzfile" or not zipfile.is_zipfile(model_path):
            weight = load_parameters(model_path)
        elif keep:  # the arrays NpzFile would give, read by 8 threads without the zip CRC pass
            weight = StreamingNpz(model_path, np.empty)
        else:  # streaming: each member's buffer recycled once uploaded (gate, up and down of a
            # layer share a size and live together: 3 per size)
            pool = l3hip.PinnedPool(keep=3, max_bytes=1 << 36) if _NPZ_READER == "pinned" else RecyclingAlloc(keep=3)
            weight = StreamingNpz(model_path, pool.empty if _NPZ_READER == "pinned" else pool)
        # every tensor the forward reads, checked before anything is allocated (the reference
        # fails late, with AttributeError on None.T, llama3.py:133-136)
        missing = [n for n in weight_names(args.n_layers) if n not in weight]
        if missing:
            raise KeyError(f"missing weight(s) {missing[:4]}{' ...' if len(missing) > 4 else ''} "
                           f"({len(missing)} of {len(weight_names(args.n_layers))})")
        self.freqs_cos, self.freqs_sin = compute_cos_sin_cache(args.dim // args.n_heads,
                                                               args.max_seq_len)
        hidden = weight.get("model.layers.0.mlp.gate_proj.weight").shape[0]
        dims = _dims(args, hidden, args.n_layers, args.vocab_size)
        if devices is not None:
            if device is not None:
                raise ValueError("pass device or devices, not both")
            self._group = l3hip.Group(dims, devices)
            self._ctx = self._group.members[0]
            tgt = self._group  # uploads go to every device; calls shard the batch rows
        else:
            self._group = None
            self._ctx = l3hip.Context(dims, DEFAULT_DEVICE if device is None else device)
            tgt = self._ctx
        self._target = tgt
        emb = weight.get("model.embed_tokens.weight")
        tgt.upload(0, l3hip.W_EMBED, emb)
        self.tok_embedding = emb if keep else _Dropped(emb.shape)
        del emb
        self.layers = [TransformerBlock(weight, i, args, _bind=(tgt, i), _keep_host=keep)
                       for i in range(args.n_layers)]
        norm_w = weight.get("model.norm.weight")
        self.norm = RMSNorm(norm_w if keep else np.array(norm_w), eps=args.norm_eps)
        tgt.upload(0, l3hip.W_FINAL_NORM, norm_w)
        lm = weight.get("lm_head.weight")
        tgt.upload(0, l3hip.W_LM_HEAD, lm)
        self.lm_head_weight = lm.T if keep else _Dropped(lm.shape[::-1])
        del lm
        tgt.finalize()
        del weight, norm_w
        if pool is not None:
            pool.clear()

    @property
    def context(self) -> l3hip.Context:
        """The device context (with ``devices=``: the first device's member context)."""
        return self._ctx

    @property
    def group(self) -> Optional[l3hip.Group]:
        """The multi-device group (``devices=``), else None."""
        return self._group

    def __call__(self, input_ids, start_pos: int):
        ids = np.asarray(input_ids)
        if ids.ndim != 2:
            raise ValueError(f"input_ids must be [B, L], got shape {ids.shape}")
        logits = self._target.forward(ids, int(start_pos))
        return logits[:, None, :]

    def generate(self, input_ids, max_new_tokens: int) -> Iterator[np.ndarray]:
        """Greedy decode with the reference's exact position schedule
        (llama3.py:310-321): prefill at 0, then decode step i >= 1 at pos = L + i,
        so KV slot L is never written and stays zero (the "decode hole").  Lazy as the
        reference's: the device may run up to 16 steps ahead of the consumer (never past
        max_new_tokens), and a schedule left early is undone before any later call."""
        ids = np.asarray(input_ids)
        _, L = ids.shape
        self._target.set_decode_horizon(max_new_tokens)
        next_id = None
        for i, curr_pos in enumerate(range(L, max_new_tokens)):
            if i == 0:
                nxt, _ = self._target.greedy_step(ids, 0)
            else:
                nxt, _ = self._target.greedy_step(next_id, curr_pos)
            next_id = nxt.reshape(-1, 1)
            yield next_id

    def generate_all(self, input_ids, max_new_tokens: int) -> np.ndarray:
        """Extension (not in the reference): the same greedy ids as ``generate`` —
        same schedule, same decode hole — computed as one device-side loop of
        graph-replayed steps with a single copy-back.  Returns int64
        ``[B, max_new_tokens - L]``.  Unlike ``generate`` it is not lazy: every step
        runs, so use it when the caller consumes all tokens.  On a multi-device model a batch of
        more than one row steps through ``Group.greedy_step`` (each device its rows, the ids
        gathered) instead of the single-device graph loop."""
        ids = np.asarray(input_ids)
        if self._group is None or self._group.n == 1 or ids.shape[0] == 1:
            return self._ctx.greedy_generate(ids, max_new_tokens)
        B, L = ids.shape
        if max_new_tokens > self.args.max_seq_len:
            raise RuntimeError(f"generate: last decode position {max_new_tokens - 1} exceeds "
                               f"max_seq_len {self.args.max_seq_len}")
        out = np.empty((B, max(0, max_new_tokens - L)), np.int64)
        nxt = None
        for i, pos in enumerate(range(L, max_new_tokens)):
            nxt, _ = self._group.greedy_step(ids if i == 0 else nxt.reshape(-1, 1), 0 if i == 0 else pos)
            out[:, i] = nxt
        return out


def main(argv=None, tokenizer_path="./tokenizer.model.np", model_path="./stories15M.model.npz"):
    """CLI of reference llama3.py:324-349: stream greedy tokens for a prompt, stop on
    EOS/BOS, then print the reference's counter line (prompt + generated tokens
    over wall time including prefill)."""
    argv = sys.argv[1:] if argv is None else argv
    prompt = argv[0] if argv else "I have a dream"
    args = ModelArgs()
    tok = Tokenizer(tokenizer_path)
    model = Llama(model_path, args)
    print(f"\n{prompt}", end="")
    ids = np.array([tok.encode(prompt)])
    count = ids.shape[1]
    t0 = time.time()
    for step in model.generate(ids, args.max_new_tokens):
        count += 1
        token = step[0].tolist()
        if token[-1] in (tok.eos_id, tok.bos_id):
            break
        print(tok.decode(token), end="")
        sys.stdout.flush()
    dt = time.time() - t0
    print(f"\n\nToken count: {count}, elapsed: {dt:.2f}s, {round(count / dt)} tokens/s")


if __name__ == "__main__":
    main()
