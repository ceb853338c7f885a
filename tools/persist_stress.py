"""Repetition check of the batch-1 persistent decode step (no fault injection): the 145-step
"I have a dream" run (llama3.py:310-321) repeated through the device loop (`generate_all`) and
the lazy `generate`, on both synthetic presets, with a second context on the same device
generating in between; every run's ids must equal the reference's fixture and no step may have
been recovered onto the graph path (`decode_recoveries` stays 0: no in-launch hand-off ever
timed out).  Prints one JSON line; exit 1 on any mismatch or recovery.

    python tools/persist_stress.py [rounds]      (default 25: 25 x (2 presets x 2 paths) runs)
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


def model_for(preset):
    g = np.load(os.path.join(REPO, "tests", "golden", f"stories15m_{preset}.npz"))
    args = synth.stories15m(1)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=int(g["seed"]), preset=preset)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        return llama3.Llama(p, args), g


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    models = {p: model_for(p) for p in ("default", "sharp")}
    runs = bad = 0
    t0 = time.perf_counter()
    for r in range(rounds):
        for preset, (m, g) in models.items():
            want = g["dream_ids"][0].tolist()
            n = int(g["dream_max_new"])
            got_all = m.generate_all(g["dream_prompt"], n)[0].tolist()
            got_lazy = [int(x[0, 0]) for x in m.generate(g["dream_prompt"], n)]
            runs += 2
            bad += (got_all != want) + (got_lazy != want)
        if r % 5 == 4:
            print(f"round {r + 1}/{rounds}: {runs} runs, {bad} mismatched", flush=True)
    rec = {p: m.context.decode_recoveries() for p, (m, _) in models.items()}
    persistent = {p: m.context.decode_persistent() for p, (m, _) in models.items()}
    out = {"runs": runs, "steps_per_run": 145, "mismatched_runs": bad, "recoveries": rec,
           "persistent": persistent, "seconds": round(time.perf_counter() - t0, 1)}
    print(json.dumps(out))
    sys.exit(1 if bad or any(rec.values()) or not all(persistent.values()) else 0)


if __name__ == "__main__":
    main()
