"""Timeline of one persistent batch-1 decode step (decode_persist.hip, L3_DECODE_PERSIST=1).

    L3_DECODE_PERSIST=1 L3_DECODE_PERSIST_STAMPS=gpurun_out/pstamps.bin python tools/persist_stamps.py

Runs a 145-step greedy loop on stories15M-shaped synthetic weights (the library dumps the last
step's stamps: [workgroup][64] s_memrealtime, 100 MHz), then prints when each stage ended
relative to the launch's earliest stamp: stage k of layer l at slot 1 + 5 l + k (QKV, attention,
O-proj, gate|up, down), 60 = the lm_head input arrived, 61 = lm_head partial published, 62 =
greedy id written (workgroup 0)."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
path = os.environ.get("L3_DECODE_PERSIST_STAMPS")
if "--read" not in sys.argv:
    import llama3  # noqa: E402
    import synth  # noqa: E402

    args = synth.stories15m(1)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        m = llama3.Llama(p, args)
    m.generate_all(np.array([[1, 76, 505, 263, 12561]]), 150)
st = np.fromfile(path, dtype=np.uint64).reshape(256, 64).astype(np.int64)
t0 = st[:, 0][st[:, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731
names = ["qkv", "attn", "oproj", "gateup", "down"]
print("workgroup 0 (a layer workgroup), stage ends in us from the launch's first stamp:")
prev = 0.0
for li in range(6):
    row = []
    for k in range(5):
        v = st[0, 1 + 5 * li + k]
        if v:
            row.append(f"{names[k]} {us(v):6.2f} (+{us(v) - prev:5.2f})")
            prev = us(v)
    print(f"  layer {li}: " + "  ".join(row))
for k, nm in ((60, "lm input"), (61, "lm partial"), (62, "greedy id")):
    if st[0, k]:
        print(f"  {nm}: {us(st[0, k]):6.2f}")
lay = st[:64]
for k in range(1, 31):
    col = lay[:, k][lay[:, k] > 0]
    if len(col):
        print(f"  slot {k:2d} {names[(k - 1) % 5]:6s} layer {(k - 1) // 5}: first {us(col.min()):6.2f} last {us(col.max()):6.2f}")
oth = st[64:]
for k in (0, 60, 61):
    col = oth[:, k][oth[:, k] > 0]
    if len(col):
        print(f"  lm workgroups slot {k}: first {us(col.min()):6.2f} last {us(col.max()):6.2f}")
