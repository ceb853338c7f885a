"""RCCL logits-gather self-test through the C ABI (l3_comm_*), N processes on one node.

    python tools/rccl_selftest.py [--world 2] [--same-device]

Each rank fills a [rows_r, VS] device buffer with rank-tagged values, the root gathers
them with l3_comm_gather_logits, and checks every row.  --same-device puts every rank on
device 0 (for a one-GPU box; RCCL may refuse duplicate devices, which is reported).
"""
import argparse
import multiprocessing as mp
import os
import sys
import traceback

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))


def rank_main(rank, world, uid, same, q):
    try:
        import l3hip

        dev = 0 if same else rank
        d = l3hip.Dims(dim=64, n_layers=0, n_heads=1, n_kv_heads=1, vocab_size=1000, hidden_dim=32,
                       max_seq_len=1, max_batch_size=1, norm_eps=1e-6)
        ctx = l3hip.Context(d, dev)
        ctx.comm_init(world, rank, uid)
        rows = [3 + r for r in range(world)]
        VS = 1000
        local = np.full((rows[rank], VS), float(rank), np.float32) + np.arange(VS, dtype=np.float32)[None] * 1e-3
        src = ctx.alloc(local.nbytes)
        ctx.h2d(src, local)
        dst = ctx.alloc(sum(rows) * VS * 4) if rank == 0 else None
        ctx.gather_logits(src, dst, rows, 0)
        ctx.synchronize()
        ok = True
        if rank == 0:
            out = np.empty((sum(rows), VS), np.float32)
            ctx.d2h(out, dst)
            off = 0
            for r in range(world):
                want = np.full((rows[r], VS), float(r), np.float32) + np.arange(VS, dtype=np.float32)[None] * 1e-3
                ok &= bool(np.array_equal(out[off:off + rows[r]], want))
                off += rows[r]
        ctx.comm_barrier()
        ctx.comm_barrier()  # repeated barriers reuse the scratch word
        ok &= ctx.comm_max(rank + 0.5) == world - 0.5  # bench.py's max-over-ranks time
        q.put((rank, ok, ""))
    except Exception:
        q.put((rank, False, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--same-device", action="store_true")
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
    import l3hip

    uid = l3hip.comm_unique_id()  # no device context needed (host-side id)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, a.world, uid, a.same_device, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(30)
    for r, ok, err in sorted(res):
        print(f"rank {r}: {'ok' if ok else 'FAIL'} {err}")
    sys.exit(0 if all(ok for _, ok, _ in res) else 1)


if __name__ == "__main__":
    main()
