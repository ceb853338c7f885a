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


@pytest.fixture(scope="module")
def c4_model():
    """BASELINE configs[3] (C4: stories15M B = 2048, L = 256), default-scale weights (the plain
    1e-4 bar applies), and a single-device model holding all 2048 rows."""
    with tempfile.TemporaryDirectory() as d:
        args = synth.stories15m(2048)
        w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=7)
        path = os.path.join(d, "c4.npz")
        synth.save_npz(path, w)
        yield args, path, w, llama3.Llama(path, args)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n", [2, 4, 8])
def test_group_virtual_c4_partition(c4_model, monkeypatch, n):
    """C4's own partition through the group on one GPU (n = 8: 256 rows per member, the 8-GPU
    node's exact split; n = 2 / 4: the strong-scaling splits of the same batch).  Every member's
    rows bit-identical to those rows run alone on one device — through the host path (each
    member's per-link 2-D copy into the caller's array, l3_group_forward_host) and through the
    device-resident gather (l3_group_forward_dev, north_star's single gather) alike — 8 spread
    rows against the live oracle within 1e-4, and the greedy step's ids equal
    (llama3.py:163-211, 285-308, 320)."""
    import llama3_oracle as orc

    monkeypatch.setenv("L3_GROUP_VIRTUAL", "1")
    args, path, w, single = c4_model
    B, L = 2048, 256
    grp = llama3.Llama(path, args, devices=[0] * n)
    g = grp.group
    VS = args.vocab_size
    ids = np.random.default_rng(2048 + n).integers(0, args.vocab_size, (B, L))
    got = np.array(grp(ids, 0))
    assert got.shape == (B, 1, VS) and np.isfinite(got).all()
    # the device-resident path: member i's ids block on its context, the gather into member 0
    ids_dev = []
    for i, m in enumerate(g.members):
        blk = np.ascontiguousarray(ids[i::n].astype(np.int32))
        p = m.alloc(blk.size * 4)
        m.h2d(p, blk)
        ids_dev.append(p)
    out_dev = g.members[0].alloc(B * VS * 4)
    g.forward_dev(ids_dev, B, L, 0, out_dev)
    g.synchronize()
    dev = np.empty((B, VS), np.float32)
    g.members[0].d2h(dev, out_dev)
    np.testing.assert_array_equal(dev, got[:, 0, :])
    g.members[0].free(out_dev)
    for m, p in zip(g.members, ids_dev):
        m.free(p)
    # greedy ids of a 3-token chunk at positions 250-252 over the caches just written
    nxt_g, _ = g.greedy_step(ids[:, 250:253], 250)
    rows = [0, 255, 256, 777, 1023, 1024, 1500, 2047]
    ref = orc.OracleModel(w, synth.stories15m(len(rows)))
    err = float(np.max(np.abs(got[rows, 0].astype(np.float64) - ref(ids[rows], 0)[:, 0])))
    assert err <= 1e-4, f"n={n}: spread rows vs the oracle max-abs {err:.3e}"
    del grp, g
    # each member's rows alone on one device: the same logits bit for bit, the same next ids
    for i in range(n):
        np.testing.assert_array_equal(got[i::n], single(ids[i::n], 0), err_msg=f"member {i} of {n}")
        nxt_s, _ = single.context.greedy_step(ids[i::n, 250:253], 250)
        np.testing.assert_array_equal(nxt_g[i::n], nxt_s, err_msg=f"member {i} greedy ids")
    print(f"C4 partition n={n}: members bit-identical (per-link host copies and the gather), "
          f"oracle max-abs {err:.2e}")


@pytest.mark.timeout(600)
def test_group_virtual_x6_members_match_single_device(model_path, single, monkeypatch):
    """The opt-in x6 GEMM path (L3_GEMM_X6=1 at context creation) through the group: at the C3
    batch each of n = 2 members prefills 128 rows x 256 positions on the x6 kernels, and its rows
    equal a single-device x6 run of those rows bit for bit (the x6 kernel's per-element
    arithmetic does not depend on M), greedy ids included."""
    monkeypatch.setenv("L3_GROUP_VIRTUAL", "1")
    monkeypatch.setenv("L3_GEMM_X6", "1")
    args, path = model_path
    n = 2
    grp = llama3.Llama(path, args, devices=[0] * n)
    single_x6 = llama3.Llama(path, args)
    ids = np.random.default_rng(7).integers(0, args.vocab_size, (256, 256))
    got = np.array(grp(ids, 0))
    nxt_g, _ = grp.group.greedy_step(ids[:, :3], 250)
    # the x6 path ran: the logits are not the fp32 kernels' bits; each path is within the parity
    # bar of the reference (test_gpu_parity.py: x6 against the oracle on these sharp weights), so
    # the two differ by at most twice it
    f32 = single(ids, 0)
    assert not np.array_equal(got, f32)
    err = np.abs(got.astype(np.float64) - f32)
    assert (err <= 2 * (1e-4 + 2e-4 * np.abs(f32))).all(), f"x6 vs fp32 max-abs {err.max():.3e}"
    for i in range(n):
        np.testing.assert_array_equal(got[i::n], single_x6(ids[i::n], 0), err_msg=f"x6 member {i}")
        nxt_s, _ = single_x6.context.greedy_step(ids[i::n, :3], 250)
        np.testing.assert_array_equal(nxt_g[i::n], nxt_s, err_msg=f"x6 member {i} greedy ids")
