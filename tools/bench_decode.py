"""Greedy-decode benchmark (BASELINE configs[0..1]): stories15M, B=1, prompt ids of
"I have a dream" = [1, 76, 505, 263, 12561], max_new_tokens=150 -> 145 greedy steps through
Llama.generate (the reference's loop, llama3.py:310-321, device argmax, ids-only D2H).

Prints one JSON line: tokens/s counted the reference's way (prompt + generated tokens over
wall time including prefill, llama3.py:347-349), per-step latency, and the ids check against
the committed golden (fixture from the reference itself).
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


PEAK_FP32_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_TBS = 8.0        # HBM3E


def step_roofline(args, B, L, steps, step_s):
    """Algorithmic work of one batched greedy step averaged over the run (llama3.py:163-211,
    304-307 at L = 1): GEMM FLOPs (QKV, O-proj, gate|up, down per layer; the lm_head), and the
    bytes a step must move at least — every weight once, each row's K / V rows 0..pos once, its
    new K / V slot written, the embedding rows — against the fp32 MFMA peak and HBM bandwidth.
    The step is bound by neither: it is ~31 dependent launches of a few us each."""
    D, H, KVH, HD, VS, nl = args.dim, args.n_heads, args.kv_heads, args.dim // args.n_heads, args.vocab_size, args.n_layers
    FD = synth.STORIES15M_HIDDEN
    qkvn = (H + 2 * KVH) * HD
    w_layer = D * qkvn + D * H * HD + D * 2 * FD + FD * D
    flops = 2.0 * B * (nl * w_layer + D * VS)
    mean_pos = L + (steps + 1) / 2.0  # decode step i at pos L + i (the reference's schedule)
    kv = nl * B * (4.0 * 2 * KVH * HD * (mean_pos + 1) + 4.0 * 2 * KVH * HD)
    weights = 4.0 * (nl * w_layer + VS * D)
    bytes_ = weights + kv + 4.0 * B * D
    tf = flops / step_s / 1e12
    tbs = bytes_ / step_s / 1e12
    floor_us = max(flops / (PEAK_FP32_TFLOPS * 1e12), bytes_ / (PEAK_HBM_TBS * 1e12)) * 1e6
    return {"flops_per_step": flops, "bytes_per_step": bytes_, "kv_bytes_per_step": kv,
            "weight_bytes_per_step": weights, "achieved_tflops": round(tf, 2),
            "mfma_frac": round(tf / PEAK_FP32_TFLOPS, 4), "achieved_tbs": round(tbs, 3),
            "hbm_frac": round(tbs / PEAK_HBM_TBS, 4), "floor_us": round(floor_us, 1),
            "step_us": round(step_s * 1e6, 1), "frac_of_floor": round(floor_us / (step_s * 1e6), 4)}


def main():
    eager = "--eager" in sys.argv  # profiling: every step eager, no device-loop leg
    if eager:
        os.environ["L3_DECODE_GRAPH"] = "0"
    if "--eager-batch" in sys.argv:  # profiling: 40 eager steps of one B-row batch
        os.environ["L3_DECODE_GRAPH"] = "0"
        B = int(sys.argv[sys.argv.index("--eager-batch") + 1])
        gb = np.load(os.path.join(REPO, "tests", "golden", "stories15m_default.npz"))
        argsb = synth.stories15m(B)
        wb = synth.make_weights(argsb, synth.STORIES15M_HIDDEN, seed=int(gb["seed"]))
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "w.npz")
            synth.save_npz(p, wb)
            mb = llama3.Llama(p, argsb)
        pr = np.random.default_rng(B).integers(3, argsb.vocab_size, (B, 5))
        t0 = time.perf_counter()
        n = sum(1 for _ in mb.generate(pr, 45))
        t = time.perf_counter() - t0
        print(json.dumps({"workload": f"stories15M greedy decode B={B} (eager)", "ms_per_step": round(t / n * 1e3, 3)}))
        return
    g = np.load(os.path.join(REPO, "tests", "golden", "stories15m_default.npz"))
    args = synth.stories15m(1)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=int(g["seed"]), preset="default")
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        model = llama3.Llama(p, args)
    prompt = g["dream_prompt"]
    list(model.generate(prompt, 20))  # warm-up (caches are overwritten by the timed run)
    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        ids = [int(x[0, 0]) for x in model.generate(prompt, int(g["dream_max_new"]))]
        runs.append(time.perf_counter() - t0)
    exact = ids == g["dream_ids"][0].tolist()
    t = float(np.median(runs))
    count = prompt.shape[1] + len(ids)
    if eager:
        print(json.dumps({"workload": "stories15M greedy decode B=1 (eager, L3_DECODE_GRAPH=0)",
                          "ms_per_step": round(t / len(ids) * 1e3, 3), "ids_exact_vs_reference": exact}))
        return
    # device-side loop (Llama.generate_all: graph replays back to back, one copy-back)
    dev = []
    for _ in range(3):
        t0 = time.perf_counter()
        all_ids = model.generate_all(prompt, int(g["dream_max_new"]))
        dev.append(time.perf_counter() - t0)
    td = float(np.median(dev))
    exact_all = all_ids[0].tolist() == g["dream_ids"][0].tolist()
    # batched device-side loop: B synthetic 5-token prompts, 145 steps
    batched = {}
    for B in (8, 64, 256):
        argsb = synth.stories15m(B)
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "w.npz")
            synth.save_npz(p, w)
            mb = llama3.Llama(p, argsb)
        pr = np.random.default_rng(B).integers(3, argsb.vocab_size, (B, prompt.shape[1]))
        mb.generate_all(pr, 20)  # warm-up + graph capture for this B
        t0 = time.perf_counter()
        out = mb.generate_all(pr, int(g["dream_max_new"]))
        tb = time.perf_counter() - t0
        steps = out.shape[1]
        batched[str(B)] = {"generated_tokens_per_s": round(out.size / tb, 1),
                           "ms_per_step": round(tb / steps * 1e3, 3),
                           "roofline": step_roofline(argsb, B, prompt.shape[1], steps, tb / steps)}
        del mb
    print(json.dumps({"workload": "stories15M greedy decode B=1, 'I have a dream', 145 steps",
                      "tokens_per_s_reference_count": round(count / t, 1),
                      "generated_tokens_per_s": round(len(ids) / t, 1),
                      "ms_per_step": round(t / len(ids) * 1e3, 3), "ids_exact_vs_reference": exact,
                      "device_loop_generated_tokens_per_s": round(len(ids) / td, 1),
                      "device_loop_ms_per_step": round(td / len(ids) * 1e3, 3),
                      "device_loop_ids_exact": exact_all,
                      "batched_device_loop": batched}))


if __name__ == "__main__":
    main()
