"""Loader probe: time ``Llama(path, args, keep_host_weights=...)`` on a
Llama-3-shape ``.npz`` slice (D 4096, FD 14336, VS 128256, ``--layers`` layers; 4 layers =
7.7 GB) for each reader (``L3_NPZ_READER``: ``utils.StreamingNpz`` into ordinary arrays — the
default — or into recycled page-locked buffers, or NumPy's NpzFile), streaming
(``keep_host_weights=False``) and with host copies kept.  Arms
alternate in one process after a warm-up read, so the file is in the page cache for all of
them (the probe measures the copy path, not the disk).  Prints one JSON line.

    python tools/load_probe.py [--layers 4] [--reps 2]
"""

import argparse
import gc
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))

import llama3  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    args = synth.llama3_shape(n_layers=a.layers, max_batch_size=1, max_seq_len=64)
    D, H, KVH, FD, VS = args.dim, args.n_heads, args.kv_heads, synth.LLAMA3_HIDDEN, args.vocab_size
    HD = D // H
    rng = np.random.default_rng(0)
    base = (rng.standard_normal(1 << 20, dtype=np.float32) * np.float32(0.02))

    def t(shape):  # cheap distinct-looking content: a tiled random block
        n = int(np.prod(shape))
        return np.resize(base, n).reshape(shape)

    w = {"model.embed_tokens.weight": t((VS, D)), "model.norm.weight": np.ones(D, np.float32),
         "lm_head.weight": t((VS, D))}
    for i in range(a.layers):
        p = f"model.layers.{i}."
        w.update({p + "self_attn.q_proj.weight": t((H * HD, D)), p + "self_attn.k_proj.weight": t((KVH * HD, D)),
                  p + "self_attn.v_proj.weight": t((KVH * HD, D)), p + "self_attn.o_proj.weight": t((D, H * HD)),
                  p + "mlp.gate_proj.weight": t((FD, D)), p + "mlp.up_proj.weight": t((FD, D)),
                  p + "mlp.down_proj.weight": t((D, FD)),
                  p + "input_layernorm.weight": np.ones(D, np.float32),
                  p + "post_attention_layernorm.weight": np.ones(D, np.float32)})
    gb = sum(v.nbytes for v in w.values()) / 1e9
    with tempfile.TemporaryDirectory(dir=os.environ.get("L3_PROBE_DIR")) as d:
        path = os.path.join(d, "slice.npz")
        t0 = time.perf_counter()
        synth.save_npz(path, w)
        write_s = time.perf_counter() - t0
        del w
        gc.collect()
        ids = np.arange(8, dtype=np.int64).reshape(1, 8)
        ref = None
        # arm -> (reader, keep_host_weights)
        arms = {"stream_threads": ("threads", False), "stream_pinned": ("pinned", False),
                "stream_npzfile": ("npzfile", False), "keep_threads": ("threads", True),
                "keep_npzfile": ("npzfile", True)}
        times = {arm: [] for arm in arms}
        for rep in range(a.reps + 1):
            for arm, (reader, keep) in arms.items():
                llama3._NPZ_READER = reader
                t0 = time.perf_counter()
                m = llama3.Llama(path, args, device=0, keep_host_weights=keep)
                dt = time.perf_counter() - t0
                out = m(ids, 0)
                if ref is None:
                    ref = out.copy()
                elif not np.array_equal(out, ref):
                    raise SystemExit(f"load_probe: {arm} logits differ from the first arm")
                del m, out
                gc.collect()
                if rep:  # rep 0 warms the page cache and the allocator
                    times[arm].append(dt)
        llama3._NPZ_READER = "threads"
    res = {"probe": "streaming .npz load, Llama-3-shape slice", "layers": a.layers, "GB": round(gb, 2),
           "write_s": round(write_s, 2)}
    for arm, v in times.items():
        s = float(np.median(v))
        res[arm] = {"s": round(s, 3), "GB/s": round(gb / s, 2), "all": [round(x, 3) for x in v]}
    res["logits_identical"] = True
    print(json.dumps(res))


if __name__ == "__main__":
    main()
