"""Determinism / batch-split check on small shapes (diagnostic): the same forward repeated, then
with 2 parts, printing max |diff| of the logits against the first run."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llama3.np_amd"))
import llama3  # noqa: E402
import synth  # noqa: E402

for (B, L) in [(2, 9), (4, 12), (2, 40), (4, 64)]:
    args = synth.tiny(max_batch_size=B)
    w = synth.make_weights(args, synth.TINY_HIDDEN, seed=3, preset="sharp")
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        m = llama3.Llama(p, args)
    ctx = m.context
    ids = np.random.default_rng(B * 100 + L).integers(0, args.vocab_size, (B, L))
    ref = m(ids, 0)
    res = []
    for parts in (1, 1, 2, 1, 2):
        ctx.set_batch_split(parts, 1)
        out = m(ids, 0)
        res.append((parts, float(np.abs(out - ref).max())))
    print(f"B={B} L={L}", res, flush=True)
