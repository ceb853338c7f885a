"""Diagnostic: repeat the pipelined forward / gather sequence of
tests/test_gpu_parity.py::test_gather_pipelined_forwards_world1 and report every
mismatch (which buffer, which rows / columns, and whose logits the wrong values are).
Also runs the same forwards with no gather at all (control).  Usage:
    python tools/gather_race_check.py [reps] [B] [L] [overlap 0|1]"""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
import l3hip  # noqa: E402
import llama3  # noqa: E402
import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = int(sys.argv[3]) if len(sys.argv) > 3 else 64
overlap = bool(int(sys.argv[4])) if len(sys.argv) > 4 else True  # l3_comm_set_overlap
args = synth.stories15m(B)
w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0)
tmp = tempfile.mkdtemp()
path = os.path.join(tmp, "m.npz")
synth.save_npz(path, w)
VS = args.vocab_size
rng = np.random.default_rng(41)
ids = [rng.integers(0, VS, (B, L)).astype(np.int32) for _ in range(3)]
ref = llama3.Llama(path, args)
want = [ref(x, 0)[:, 0, :] for x in ids]
m = llama3.Llama(path, args)
ctx = m.context
ctx.comm_init(1, 0, l3hip.comm_unique_id())
ctx.set_comm_overlap(overlap)
ids_dev = [ctx.alloc(x.nbytes) for x in ids]
for d, x in zip(ids_dev, ids):
    ctx.h2d(d, x)
buf = ctx.alloc(B * VS * 4)
dst = [ctx.alloc(B * VS * 4) for _ in range(2)]
bad = 0
for rep in range(reps):
    for mode in ("gather", "control"):
        for parts in (1, 2):
            ctx.set_batch_split(parts, min_tokens=1)
            for k in range(3):
                ctx.forward_dev(ids_dev[k], B, L, 0, buf)
                if k < 2 and mode == "gather":
                    ctx.gather_logits(buf, dst[k], [B], root=0)
            names = ("dst0", "dst1", "buf") if mode == "gather" else ("buf",)
            ptrs = (dst[0], dst[1], buf) if mode == "gather" else (buf,)
            wants = want if mode == "gather" else want[2:]
            for nm, p, wt in zip(names, ptrs, wants):
                g = ctx.d2h(np.empty((B, VS), np.float32), p)
                ne = g != wt
                if ne.any():
                    bad += 1
                    r, c = np.nonzero(ne)
                    whose = [int(np.isclose(g[ne], x[ne]).mean() * 100) for x in want]
                    print(f"rep {rep} {mode} parts {parts} {nm}: {ne.sum()} wrong, rows "
                          f"{sorted(set(r.tolist()))}, cols {c.min()}..{c.max()}, "
                          f"% matching step 0/1/2: {whose}", flush=True)
print(f"done: {reps} reps (overlap {overlap}), {bad} bad buffers", flush=True)
