"""Where the drop-in host path's time goes (C3: Llama.__call__ on host ids, pinned logits back)
against the device-resident forward: forward alone, forward + host path, a bare 32.8 MB D2H into
pinned memory, the int64 ids upload alone.  Prints one JSON line.

    python tools/host_path_probe.py
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
import l3hip  # noqa: E402
import llama3  # noqa: E402
import synth  # noqa: E402


def timeit(fn, n):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    B, L = 256, 256
    args = synth.stories15m(B)
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=0)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "w.npz")
        synth.save_npz(p, w)
        m = llama3.Llama(p, args)
    ctx = m.context
    VS = args.vocab_size
    ids = np.random.default_rng(1).integers(0, VS, (B, L))
    ids_dev = ctx.alloc(B * L * 4)
    ctx.h2d(ids_dev, ids.astype(np.int32))
    out_dev = ctx.alloc(B * VS * 4)

    def dev():
        ctx.forward_dev(ids_dev, B, L, 0, out_dev)
        ctx.synchronize()

    def host():
        x = m(ids, 0)
        del x

    pin = l3hip.pinned.empty((B, VS), np.float32)

    def d2h():
        ctx.d2h(pin, out_dev)

    ids32 = ids.astype(np.int32)

    def h2d():
        ctx.h2d(ids_dev, ids32)

    res = {"forward_dev_ms": round(timeit(dev, 10), 4), "host_path_ms": round(timeit(host, 10), 4),
           "d2h_32.8MB_ms": round(timeit(d2h, 10), 4), "h2d_ids_ms": round(timeit(h2d, 10), 4)}
    res["d2h_GBps"] = round(B * VS * 4 / res["d2h_32.8MB_ms"] / 1e6, 1)
    # the later batch part's last k layers wait for part 0's (L3_HOST_LAG, runtime.hip
    # forward_dev): part 0's logits copy starts while part 1 still computes; interleaved rounds
    lags = [int(x) for x in os.environ.get("PROBE_LAGS", "0,1,2,3").split(",")]
    for rnd in range(2):
        for k in lags:
            os.environ["L3_HOST_LAG"] = str(k)
            res[f"host_path_lag{k}_ms_r{rnd}"] = round(timeit(host, 20), 4)
    os.environ.pop("L3_HOST_LAG", None)
    x = m(ids, 0)
    for k in lags:  # every lag returns the same logits
        os.environ["L3_HOST_LAG"] = str(k)
        res[f"lag{k}_bitwise_equal"] = bool(np.array_equal(m(ids, 0), x))
    os.environ.pop("L3_HOST_LAG", None)
    # more batch parts on the host path (a staircase of lags: the last part's copy is smaller)
    for rnd in range(2):
        for parts, k in ((2, 2), (3, 2), (4, 2), (3, 1), (4, 1)):
            ctx.set_batch_split(parts)
            os.environ["L3_HOST_LAG"] = str(k)
            res[f"host_path_parts{parts}_lag{k}_ms_r{rnd}"] = round(timeit(host, 20), 4)
    for parts in (3, 4):
        ctx.set_batch_split(parts)
        res[f"forward_dev_parts{parts}_ms"] = round(timeit(dev, 10), 4)
    os.environ.pop("L3_HOST_LAG", None)
    ctx.set_batch_split(2)
    ctx.set_batch_split(1)
    res["forward_dev_split1_ms"] = round(timeit(dev, 10), 4)
    res["host_path_split1_ms"] = round(timeit(host, 10), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
