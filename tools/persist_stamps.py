"""Timeline of one persistent batch-1 decode step (decode_persist.hip, L3_DECODE_PERSIST=1).

    L3_DECODE_PERSIST=1 L3_DECODE_PERSIST_STAMPS=gpurun_out/pstamps.bin python tools/persist_stamps.py

Runs a 145-step greedy loop on stories15M-shaped synthetic weights (the library dumps the last
step's stamps: [workgroup][128] s_memrealtime, 100 MHz), then prints, per stage, when its input
arrived (slot 1 + 10 l + 2 k) and its output was published (2 + 10 l + 2 k) relative to the
launch's earliest stamp; 100-105 the lm_head and the final argmax."""
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
    # --max-new N: e.g. 143 = 5 + 2 eager steps + 17 graphs of 8 (the last launch a multi-step one)
    max_new = int(sys.argv[sys.argv.index("--max-new") + 1]) if "--max-new" in sys.argv else 150
    m.generate_all(np.array([[1, 76, 505, 263, 12561]]), max_new)
st = np.fromfile(path, dtype=np.uint64).reshape(256, 128).astype(np.int64)
xcc = st[:, 127].copy()
st[:, 127] = 0
t0 = st[:, 0][st[:, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731
names = ["qkv", "attn", "oproj", "gateup", "down"]
lay_idx = np.arange(64)  # layer workgroups (GL = 64; fold: 0..5 the heads)
lm_idx = np.setdiff1d(np.arange(256), lay_idx)
lay = st[lay_idx]


def span(rows, k):
    col = rows[:, k][rows[:, k] > 0]
    return (us(col.min()), us(col.max())) if len(col) else (None, None)


print("layer workgroups: per stage, input arrived (first..last) -> output published (first..last), us")
for li in range(6):
    for k in range(5):
        a0, a1 = span(lay, 1 + 10 * li + 2 * k)
        p0, p1 = span(lay, 2 + 10 * li + 2 * k)
        if p0 is None:
            continue
        arr = f"{a0:7.2f}..{a1:7.2f}" if a0 is not None else " " * 16
        print(f"  L{li} {names[k]:6s} in {arr}  out {p0:7.2f}..{p1:7.2f}")
for k, nm in ((0, "start"), (100, "lm input"), (103, "lm rms"), (104, "lm rows done"), (101, "lm partial")):
    a = span(lay, k)
    b = span(st[lm_idx], k)
    print(f"  {nm:12s} layer wgs {a[0]}..{a[1]}   lm wgs {b[0]}..{b[1]}")
print("attention workgroups, layer 1: in / scores / max / sum / PV / part stored / out")
for h in range(6):
    print("  head", h, " ".join(f"{us(st[lay_idx[h], k]):7.2f}" for k in (13, 110, 111, 112, 113, 114, 14)))
print("layer workgroups' XCDs:", sorted(set(xcc[lay_idx].tolist())), " lm workgroups' XCDs:", sorted(set(xcc[lm_idx].tolist())))
if st[0, 120] > 0:
    print("fold head workgroups, layer 1: h2 in / QKV dot done / K, V requested + barrier / RoPE done / attention in")
    for h in range(6):
        print("  head", h, " ".join(f"{us(st[h, k]):7.2f}" for k in (11, 120, 121, 122, 13)))
for k, nm in ((105, "wg0 partials in"), (102, "greedy id")):
    print(f"  {nm}: {us(st[0, k]):.2f}")
