"""x6 path: C3 forwards repeated with the batch split on and off, bitwise comparisons.

    python tools/x6_determinism.py [--fp32] [--dev]
(--fp32: the default GEMM path as the control; --dev: l3_forward_dev instead of Llama.__call__)
"""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "llama3.np_amd"), os.path.join(REPO, "tests")]
import llama3  # noqa: E402
import synth  # noqa: E402

args = synth.stories15m(256)
w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0, preset="default")
with tempfile.TemporaryDirectory() as d:
    path = os.path.join(d, "w.npz")
    synth.save_npz(path, w)
    m = llama3.Llama(path, args)
ids = np.random.default_rng(1).integers(0, args.vocab_size, (256, 256))
ctx = m.context
ctx.set_gemm_x6("--fp32" not in sys.argv)
if "--dev" in sys.argv:
    ids_dev = ctx.alloc(ids.size * 4)
    ctx.h2d(ids_dev, ids.astype(np.int32))
    lg = ctx.alloc(256 * args.vocab_size * 4)

    def run():
        ctx.forward_dev(ids_dev, 256, 256, 0, lg)
        out = np.empty((256, args.vocab_size), np.float32)
        ctx.d2h(out, lg)
        return out
else:
    def run():
        return m(ids, 0)
outs = {}
for split in (2, 1, 2, 1, 2):
    ctx.set_batch_split(split)
    outs.setdefault(split, []).append(run())
tag = " ".join(a for a in sys.argv[1:]) or "x6 host"
for split, o in outs.items():
    same = [bool(np.array_equal(o[0], x)) for x in o[1:]]
    print(f"[{tag}] split {split}: repeats bit-identical {same}", flush=True)
d = np.abs(outs[1][0] - outs[2][0].reshape(outs[1][0].shape))
print(f"[{tag}] split 1 vs 2: identical {bool((d == 0).all())}, differing {(d > 0).mean():.4%}, max {d.max():.3e}")
