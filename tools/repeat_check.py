"""Run-to-run determinism at full size (no fault injection): the same input through the same
context many times must give bit-identical outputs — the forward has no atomics in its
arithmetic and a fixed reduction order, whatever the two batch-part streams' interleaving.

    python tools/repeat_check.py c3 [reps]        C3 prefill (B=256, L=256), logits of every rep
                                                  against the first (default 50 reps)
    python tools/repeat_check.py batched [reps]   batched device loop (B=256, 5-token prompts,
                                                  145 steps), ids of every rep against the first

Parity of the first output with the reference is the tests' job (tests/test_gpu_parity.py); this
pins that the answer does not move between runs.  Prints one JSON line; exit 1 on a difference.
"""
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


def model(B):
    args = synth.stories15m(B)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        return llama3.Llama(p, args), args


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "c3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    m, args = model(256)
    rng = np.random.default_rng(1)
    t0 = time.perf_counter()
    diff = 0
    if mode == "c3":
        ids = rng.integers(0, args.vocab_size, (256, 256))
        first = np.array(m(ids, 0), copy=True)
        for _ in range(reps - 1):
            diff += int(not np.array_equal(m(ids, 0), first))
        what = "C3 logits [256, 1, 32000]"
    elif mode == "batched":
        prompt = rng.integers(3, args.vocab_size, (256, 5))
        first = m.generate_all(prompt, 150)
        for _ in range(reps - 1):
            diff += int(not np.array_equal(m.generate_all(prompt, 150), first))
        what = "batched device loop ids [256, 145]"
    else:
        raise SystemExit(f"unknown mode {mode}")
    print(json.dumps({"mode": mode, "compared": what, "reps": reps, "differing_reps": diff,
                      "finite": bool(np.isfinite(first).all()), "seconds": round(time.perf_counter() - t0, 1)}))
    sys.exit(1 if diff else 0)


if __name__ == "__main__":
    main()
