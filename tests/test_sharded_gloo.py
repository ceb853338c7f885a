"""Multi-rank batch-sharded prefill, rehearsed on CPU with gloo (world sizes 2 and 3).

The GPU path (ShardedPrefill.on_device) runs the HIP forward per rank and gathers logits
with RCCL; here the same ShardedPrefill control flow runs with the oracle as the per-rank
forward and a gloo gather as the transport — test infrastructure standing in for the two
device operations — and rank 0 checks the assembled [B, 1, VS] against one unsharded oracle
forward (bit-exact: rows are independent in the reference, llama3.py:163-211).
"""

import os
import socket
import sys

import numpy as np
import pytest

from sharded import ShardedPrefill, rows_per_rank, shard_rows


def test_shard_rows_partition():
    for B in (1, 2, 5, 8, 256, 2048, 257):
        for world in (1, 2, 3, 4, 8):
            blocks = [shard_rows(B, world, r) for r in range(world)]
            assert sum(n for _, n in blocks) == B
            pos = 0
            for s, n in blocks:  # contiguous, in rank order
                assert s == pos
                pos += n
            assert max(n for _, n in blocks) - min(n for _, n in blocks) <= 1
    assert rows_per_rank(2048, 8) == [256] * 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, outdir):
    import torch.distributed as dist

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "llama3.np_amd"), os.path.join(os.path.dirname(here), "oracle")):
        sys.path.insert(0, p)
    import llama3_oracle as orc
    import synth
    from sharded import ShardedPrefill

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = synth.tiny(8)
    w = synth.make_weights(args, synth.TINY_HIDDEN, seed=5, preset="sharp")
    model = orc.OracleModel(w, args)  # this rank's replica (own caches)

    def forward_local(ids, start_pos):
        return model(ids, start_pos)[:, 0, :]

    def gather(local, counts):
        objs = [None] * world if rank == 0 else None
        dist.gather_object(local, objs, dst=0)
        if rank != 0:
            return None
        return np.concatenate([o for o in objs if o is not None], axis=0)

    def gather_ids(local, counts):  # the device path's per-rank argmax, then an ids gather
        mine = None if local is None else np.argmax(local, axis=-1)
        objs = [None] * world if rank == 0 else None
        dist.gather_object(mine, objs, dst=0)
        if rank != 0:
            return None
        return np.concatenate([o for o in objs if o is not None], axis=0)

    sp = ShardedPrefill(world, rank, forward_local, gather, gather_ids=gather_ids)
    results = []
    for B, L, start in cases:
        ids = np.random.default_rng(B * 100 + L).integers(0, args.vocab_size, (B, L))
        out = sp(ids, start)
        if rank == 0:
            ref = orc.OracleModel(w, args)
            if start:
                ref(np.random.default_rng(1).integers(0, args.vocab_size, (B, start)), 0)
            want = ref(ids, start)
            results.append(bool(np.array_equal(out, want)) and out.shape == (B, 1, args.vocab_size))
        else:
            assert out is None
        # greedy ids only (SURVEY 8(e) option): the same rows' argmax, ids gathered
        nxt = sp.greedy(ids, start)
        if rank == 0:
            results.append(nxt.shape == (B, 1) and nxt.dtype == np.int64
                           and bool(np.array_equal(nxt[:, 0], np.argmax(want[:, 0, :], axis=-1))))
        else:
            assert nxt is None
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        np.save(os.path.join(outdir, "ok.npy"), np.array(results))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_prefill_gloo(world, tmp_path):
    mp = pytest.importorskip("torch.multiprocessing")
    cases = [(4, 7, 0), (5, 3, 0), (1, 6, 0)]  # even, uneven (3+2 / 2+2+1), one rank empty
    mp.spawn(_worker, args=(world, _free_port(), cases, str(tmp_path)), nprocs=world, join=True)
    ok = np.load(tmp_path / "ok.npy")
    assert ok.all(), ok


def _uid_worker(rank, world, key, outdir):
    import l3hip

    l3hip.comm_unique_id = lambda: bytes(range(7, 135))  # stand-in id (no RCCL bootstrap)
    uid = l3hip.exchange_unique_id(rank, world, key, timeout_s=30)
    with open(os.path.join(outdir, f"uid{rank}"), "wb") as f:
        f.write(uid)


def test_unique_id_file_exchange(tmp_path):
    """bench.py's torch-free RCCL id hand-off: every rank reads rank 0's 128 bytes."""
    import multiprocessing as mp

    key = f"test_{os.getpid()}_{_free_port()}"
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_uid_worker, args=(r, 3, key, str(tmp_path))) for r in (2, 1, 0)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    got = [(tmp_path / f"uid{r}").read_bytes() for r in range(3)]
    assert got[0] == bytes(range(7, 135)) and got[1] == got[0] and got[2] == got[0]
    os.remove(os.path.join("/tmp", f"l3_rccl_uid_{key}"))


def test_greedy_needs_gather_ids():
    """ShardedPrefill.greedy (ids-only gather) refuses when built without gather_ids, and
    checks the input rank like __call__."""
    sp = ShardedPrefill(1, 0, lambda ids, s: ids, lambda local, counts: local)
    with pytest.raises(NotImplementedError):
        sp.greedy(np.zeros((2, 3), np.int64), 0)
    sp = ShardedPrefill(1, 0, lambda ids, s: np.eye(4)[ids[:, -1]],
                        lambda local, counts: local,
                        gather_ids=lambda local, counts: np.argmax(local, axis=-1))
    np.testing.assert_array_equal(sp.greedy(np.array([[0, 3], [1, 2]]), 0), [[3], [2]])
    with pytest.raises(ValueError):
        sp.greedy(np.zeros(3, np.int64), 0)
