"""Timeline of one persistent batched decode step (decode_batch.hip, B rows).

    L3_DECODE_PERSIST_STAMPS=gpurun_out/bstamps.bin python tools/pbatch_stamps.py [B]

Runs a 145-step greedy loop at batch B (default 256) on stories15M-shaped synthetic weights; the
library dumps the last step's stamps ([workgroup][128] s_memrealtime, 100 MHz).  Per layer and
stage: when the workgroups had their input (first..last) and finished (first..last), in us from
the launch's earliest stamp."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
path = os.environ.get("L3_DECODE_PERSIST_STAMPS")
B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] != "--read" else 256
if "--read" not in sys.argv:
    import llama3  # noqa: E402
    import synth  # noqa: E402

    args = synth.stories15m(B)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        m = llama3.Llama(p, args)
    prompt = np.random.default_rng(0).integers(3, args.vocab_size, (B, 5))
    m.generate_all(prompt, 150)
st = np.fromfile(path, dtype=np.uint64).reshape(256, 128).astype(np.int64)
act = st[:, 1] > 0
t0 = st[:, 0][st[:, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731


def span(k):
    col = st[act, k]
    col = col[col > 0]
    return (us(col.min()), us(col.max())) if len(col) else (float("nan"), float("nan"))


print(f"B={B}: {int(act.sum())} layer workgroups; start {span(0)}")
names = [("qkv in", 1), ("qkv out", 2), ("attn in", 3), ("attn out", 4), ("o in", 5), ("o out", 6),
         ("gu in", 7), ("gu out", 8), ("down in", 9), ("down out", 10)]
for li in range(6):
    print(f"L{li} " + "  ".join(f"{n} {span(k + 10 * li)[0]:6.1f}..{span(k + 10 * li)[1]:6.1f}" for n, k in names))
