"""The single-process multi-device group (l3_group_*, runtime.hip) with n > 1 members, run on the
one-GPU box: L3_GROUP_VIRTUAL=1 lets n member contexts share device 0 and turns only the grouped
ncclSend / ncclRecv into device copies into the same member-0 buffers.  The row split (row r on
member r % n as its local row r // n), uneven member row counts (members with no rows
included), the peer-buffer offsets, the 2-D row interleave and the ids-only greedy gather all
execute for real; the RCCL point-to-point calls are the only group code left for the 8-GPU node.

Reference: llama3.py:163-211 (rows never interact), 285-308 (the forward returns every row's
last-position logits), 316-320 (greedy ids).  Each member computes its rows as a single-device
context computes the same rows as a batch of their own, so the group's rows i, i + n, ... are
compared bit for bit with a single-device Llama run on exactly those rows, and the whole batch
with the single-device batch within the parity bar (another batch size may take another GEMM
kernel, which rounds differently).
"""

import os
import tempfile

import numpy as np
import pytest

import llama3
import synth

pytestmark = pytest.mark.gpu

MAXB = 256


@pytest.fixture(scope="module")
def model_path():
    with tempfile.TemporaryDirectory() as d:
        args = synth.stories15m(MAXB)
        path = os.path.join(d, "w.npz")
        synth.save_npz(path, synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=4, preset="sharp"))
        yield args, path


@pytest.fixture(scope="module")
def single(model_path):
    args, path = model_path
    return llama3.Llama(path, args)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [2, 3, 8])
def test_group_virtual_members_match_single_device(model_path, single, monkeypatch, n):
    monkeypatch.setenv("L3_GROUP_VIRTUAL", "1")
    args, path = model_path
    grp = llama3.Llama(path, args, devices=[0] * n)
    assert grp.group is not None and grp.group.n == n
    rng = np.random.default_rng(100 + n)
    for B, L in ((5, 40), (6, 40), (64, 40), (256, 256)):  # 256 x 256: the C3 batch
        ids = rng.integers(0, args.vocab_size, (B, L))
        got = grp(ids, 0)
        assert got.shape == (B, 1, args.vocab_size)
        got = np.array(got)
        # greedy ids of the next 3-token chunk on the caches just written (C3: a greedy prefill)
        chunk, at = (ids[:, :3], L) if L + 3 <= args.max_seq_len else (ids, 0)
        nxt_g, _ = grp.group.greedy_step(chunk, at)
        # each member's rows against the same rows as a single-device batch of their own
        for i in range(n):
            rows = ids[i::n]
            if rows.shape[0] == 0:
                continue
            want = single(rows, 0)
            np.testing.assert_array_equal(got[i::n], want, err_msg=f"B={B} member {i} of {n}")
            nxt_s, _ = single.context.greedy_step(chunk[i::n], at)
            np.testing.assert_array_equal(nxt_g[i::n], nxt_s, err_msg=f"B={B} member {i} greedy ids")
        # the whole batch against the single-device batch (parity bar; sharp preset: rtol form)
        full = single(ids, 0)
        err = np.abs(got.astype(np.float64) - full)
        assert (err <= 1e-4 + 2e-4 * np.abs(full)).all(), f"B={B}: max-abs {err.max():.3e}"
        print(f"n={n} B={B} L={L}: members bit-identical to their rows alone; vs the whole batch max-abs {err.max():.2e}")
    # one prompt: member 0's own single-device path (graph-replayed decode)
    p = rng.integers(0, args.vocab_size, (1, 6))
    np.testing.assert_array_equal(grp.generate_all(p, 40), single.generate_all(p, 40))
    # a batched greedy loop through the group (ids gathered each step) equals the single device's
    pb = rng.integers(0, args.vocab_size, (5, 6))
    np.testing.assert_array_equal(grp.generate_all(pb, 30), single.generate_all(pb, 30))
