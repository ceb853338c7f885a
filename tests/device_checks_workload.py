"""Workload for tests/test_gpu_device_checks.py, run in its own process with L3_LIB_PATH set to
the device bounds-check build (libllama3hip_check.so): the plumbing self-test, then every
kernel family the library launches — tiled / skinny / GEMV / split-free GEMMs with every
epilogue, prefill and decode attention, the argmax kernels, the persistent batch-1 step, the
captured batched steps, the K / V undo of an abandoned run-ahead — up to the last cache slot.
Prints one JSON line: the check build's counts after the self-test and after the workload."""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "llama3.np_amd"))
import llama3  # noqa: E402
import synth  # noqa: E402


def main():
    out = {}
    with tempfile.TemporaryDirectory() as d:
        args = synth.stories15m(16)
        args.max_seq_len = 300
        w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=3, preset="sharp")
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        m = llama3.Llama(p, args)
    ctx = m.context
    out["enabled"], _ = ctx.device_check_counts()
    ctx.device_check_selftest()
    out["selftest"] = ctx.device_check_counts()[1]
    out["after_selftest_read"] = ctx.device_check_counts()[1]  # cleared by the read
    rng = np.random.default_rng(4)
    # prefill: tiled GEMMs and the prefill attention (T = 16 x 256), a chunk at start_pos 256,
    # short prompts on the skinny kernel
    ids = rng.integers(0, args.vocab_size, (16, 256))
    m(ids, 0)
    m(rng.integers(0, args.vocab_size, (16, 40)), 256)
    m(rng.integers(0, args.vocab_size, (4, 3)), 0)
    # eager L = 1 steps: GEMV (B <= 8) and skinny (B = 16) decode, up to the last slot (299)
    for B, pos in ((8, 296), (16, 297), (1, 298), (16, 299)):
        m(rng.integers(0, args.vocab_size, (B, 1)), pos)
    # captured steps: batch 1 (persistent), B = 3 and B = 16 (argmax partials), to the end
    prompt = rng.integers(0, args.vocab_size, (1, 5))
    m.generate_all(prompt, args.max_seq_len)
    m.generate_all(rng.integers(0, args.vocab_size, (3, 7)), 60)
    m.generate_all(rng.integers(0, args.vocab_size, (16, 5)), args.max_seq_len)
    # lazy generate dropped after a few steps, then an off-schedule call: the run-ahead's K / V
    # slots are restored (kv_restore)
    g = m.generate(prompt, 120)
    for _ in range(3):
        next(g)
    del g
    m(rng.integers(0, args.vocab_size, (1, 4)), 0)
    out["workload"] = ctx.device_check_counts()[1]
    out["persistent"] = ctx.decode_persistent()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
