"""Batch-sharded prefill across the GPUs of one node.

The reference's forward never mixes batch rows (``llama3.py:163-211``: every op is
per row except the weights), so the batch axis shards with no exchange until the
very end: rank r runs ``Llama.__call__`` on its contiguous block of rows and one
gather brings the ``[B_r, VS]`` last-position logits to the root — an RCCL
point-to-point gather over xGMI inside ``libllama3hip`` (``l3_comm_gather_logits``:
root posts one ``ncclRecv`` per peer, peers one ``ncclSend``, all in one group).
Weights are replicated (98 MB for stories15M); each rank keeps its own KV cache
for its rows.  Single-prompt greedy decode stays on one GPU (replica).

``ShardedPrefill`` holds only the partitioning / assembly logic and takes the two
operations it needs as callables, so the multi-rank control flow is testable on
CPU with gloo (tests/test_sharded_gloo.py); ``ShardedPrefill.on_device`` wires
them to the HIP context (device-resident logits, RCCL gather, one D2H on root).
"""

from typing import Callable, List, Optional, Tuple

import numpy as np


def shard_rows(B: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous row block of ``rank``: the first ``B % world`` ranks take one extra row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(B, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def rows_per_rank(B: int, world: int) -> List[int]:
    return [shard_rows(B, world, r)[1] for r in range(world)]


class ShardedPrefill:
    """Prefill ``input_ids [B, L]`` with rows split over ``world`` ranks.

    forward_local(ids_block, start_pos) -> local logits handle (whatever ``gather`` takes)
    gather(local, counts) -> full logits [B, VS] on the root, None elsewhere
    gather_ids(local, counts) -> (optional) greedy ids [B] on the root, None elsewhere: each
        rank's argmax over its own rows, only the ids cross the links (SURVEY 8(e) option)
    """

    def __init__(self, world: int, rank: int, forward_local: Callable, gather: Callable,
                 root: int = 0, gather_ids: Optional[Callable] = None):
        self.world, self.rank, self.root = world, rank, root
        self.forward_local = forward_local
        self.gather = gather
        self.gather_ids = gather_ids

    def __call__(self, input_ids, start_pos: int) -> Optional[np.ndarray]:
        ids = np.asarray(input_ids)
        if ids.ndim != 2:
            raise ValueError(f"input_ids must be [B, L], got {ids.shape}")
        B = ids.shape[0]
        start, n = shard_rows(B, self.world, self.rank)
        local = self.forward_local(ids[start:start + n], start_pos) if n else None
        full = self.gather(local, rows_per_rank(B, self.world))
        return None if full is None else full[:, None, :]

    def greedy(self, input_ids, start_pos: int) -> Optional[np.ndarray]:
        """Next greedy ids int64 ``[B, 1]`` on the root — ``np.argmax`` of the last-position
        logits (llama3.py:320) — with only B ids gathered instead of B x VS logits; None
        elsewhere."""
        if self.gather_ids is None:
            raise NotImplementedError("this ShardedPrefill was built without gather_ids")
        ids = np.asarray(input_ids)
        if ids.ndim != 2:
            raise ValueError(f"input_ids must be [B, L], got {ids.shape}")
        B = ids.shape[0]
        start, n = shard_rows(B, self.world, self.rank)
        local = self.forward_local(ids[start:start + n], start_pos) if n else None
        full = self.gather_ids(local, rows_per_rank(B, self.world))
        return None if full is None else np.asarray(full, dtype=np.int64).reshape(B, 1)

    @classmethod
    def on_device(cls, model, world: int, rank: int,
                  bcast_uid: Optional[Callable[[Optional[bytes]], bytes]] = None, root: int = 0):
        """Wire to a ``llama3.Llama`` on this rank's GPU.  ``bcast_uid`` ships the
        128-byte RCCL id from the root to every rank (any host-side channel); by default a
        file hand-off in /tmp keyed by ``l3hip.launch_key()`` (one node)."""
        import l3hip

        ctx = model.context
        VS = ctx.dims.vocab_size
        if bcast_uid is None:
            if root != 0:
                raise ValueError("the default id exchange needs root 0")
            key = l3hip.launch_key()
            uid = l3hip.exchange_unique_id(rank, world, key)
        else:
            uid = bcast_uid(l3hip.comm_unique_id() if rank == root else None)
        ctx.comm_init(world, rank, uid)
        if bcast_uid is None and rank == 0:
            l3hip.remove_unique_id(key)
        bufs = {}

        def buffer(name, nbytes):
            if bufs.get(name, (0, 0))[1] < nbytes:
                if name in bufs:
                    ctx.free(bufs[name][0])
                bufs[name] = (ctx.alloc(nbytes), nbytes)
            return bufs[name][0]

        def forward_local(ids_block, start_pos):
            ids32 = np.ascontiguousarray(ids_block, dtype=np.int64)
            if ids32.size and (ids32.min() < -VS or ids32.max() >= VS):
                raise IndexError("token id out of range")
            ids32 = np.where(ids32 < 0, ids32 + VS, ids32).astype(np.int32)
            n, L = ids32.shape
            d_ids = buffer("ids", ids32.nbytes)
            ctx.h2d(d_ids, ids32)
            d_out = buffer("logits", n * VS * 4)
            ctx.forward_dev(d_ids, n, L, start_pos, d_out)
            return d_out

        def gather(local, counts):
            total = sum(counts)
            dst = buffer("gathered", total * VS * 4) if rank == root else None
            src = local if local is not None else buffer("empty", 4)
            ctx.gather_logits(src, dst, counts, root)
            if rank != root:
                ctx.synchronize()
                return None
            out = np.empty((total, VS), np.float32)
            return ctx.d2h(out, dst)

        def gather_ids(local, counts):
            total = sum(counts)
            dst = buffer("gathered_ids", total * 4) if rank == root else None
            src = local if local is not None else buffer("empty", 4)
            ctx.gather_argmax(src, dst, counts, root)
            if rank != root:
                ctx.synchronize()
                return None
            return ctx.d2h(np.empty(total, np.int32), dst)

        return cls(world, rank, forward_local, gather, root, gather_ids)
