"""The persistent batch-1 decode step (decode_persist.hip) as every batch-1 user's default path:
values pinned against the reference, not only ids; the launch gated on the device it runs on;
a step that gives up on an in-launch hand-off recovered on the 25-kernel graph path with the
reference's result; the HD = 64 instance.

Reference: llama3.py:304-321 (final norm, lm_head, greedy argmax, the generate schedule with
its decode hole).  Fixtures: tests/golden/stories15m_{default,sharp}.npz, made by running the
reference itself (tests/golden/make_golden.py): 145 greedy ids of "I have a dream", and per
step the winning logit (dream_max) and the top-2 margin (dream_margin).
"""

import os
import tempfile

import numpy as np
import pytest

import llama3
import llama3_oracle as orc
import synth
from config import ModelArgs
from conftest import load_golden

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 2e-4  # north star 1e-4; the sharp preset: the reference test's own form


@pytest.fixture(scope="module")
def tmpdir_mod():
    with tempfile.TemporaryDirectory() as d:
        yield d


def _stories(tmp, preset):
    g = load_golden(f"stories15m_{preset}")
    args = synth.stories15m(1)
    path = os.path.join(tmp, f"s15_{preset}.npz")
    if not os.path.exists(path):
        synth.save_npz(path, synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=int(g["seed"]), preset=preset))
    return g, args, path


def _dream(g):
    return (np.asarray(g["dream_prompt"]).reshape(1, -1), np.asarray(g["dream_ids"]).reshape(1, -1),
            int(g["dream_max_new"]))


@pytest.mark.parametrize("persist", ["1", "0"])
@pytest.mark.parametrize("preset", ["default", "sharp"])
def test_decode_values_match_reference(tmpdir_mod, monkeypatch, preset, persist):
    """Each greedy step's winning logit (the value np.argmax picked, llama3.py:320) against the
    reference's, over all 145 steps: the persistent step (one launch per step, values from its
    lm_head partials) and the 25-kernel graph (values from its argmax kernels), in the device
    loop.  Default preset: within 1e-4; sharp (|logits| ~ 33): 1e-4 + 2e-4 |ref|.  Reports the
    smallest top-2 margin of the run (the reference's), i.e. how close an id came to flipping."""
    monkeypatch.setenv("L3_DECODE_PERSIST", persist)
    g, args, path = _stories(tmpdir_mod, preset)
    prompt, want, n = _dream(g)
    m = llama3.Llama(path, args)
    ids, vals = m.context.greedy_generate(prompt, n, values=True)
    np.testing.assert_array_equal(ids, want)
    assert m.context.decode_persistent() == (persist == "1")
    ref = np.asarray(g["dream_max"]).reshape(1, -1)
    err = np.abs(vals.astype(np.float64) - ref)
    tol = ATOL + (RTOL * np.abs(ref) if preset == "sharp" else 0.0)
    assert (err <= tol).all(), f"worst step {int(err.argmax())}: {err.max():.3e}"
    margin = np.asarray(g["dream_margin"])
    print(f"{preset} persist={persist}: max-abs {err.max():.2e} over {ref.size} steps, "
          f"|logit| <= {np.abs(ref).max():.2f}, smallest top-2 margin {margin.min():.2e} at step {int(margin.argmin())}")
    # the ids-only entry point is the same loop
    m2 = llama3.Llama(path, args)
    np.testing.assert_array_equal(m2.generate_all(prompt, n), want)


def test_persistent_decode_needs_its_cus(tmpdir_mod, monkeypatch):
    """A device with fewer CUs than the step's layer + lm workgroups (a CPX partition has 32;
    L3_DECODE_PERSIST_MAX_CUS=32 makes this device look like one) captures the 25-kernel graph
    instead of failing: the device loop, the lazy generator and an abandoned generator all give
    the reference's 145 ids."""
    g, args, path = _stories(tmpdir_mod, "default")
    prompt, want, n = _dream(g)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    monkeypatch.setenv("L3_DECODE_PERSIST_MAX_CUS", "32")
    m = llama3.Llama(path, args)
    np.testing.assert_array_equal(m.generate_all(prompt, n), want)
    assert not m.context.decode_persistent()
    np.testing.assert_array_equal(np.concatenate(list(m.generate(prompt, n)), axis=1), want)
    assert not m.context.decode_persistent()
    # with every CU visible again the next capture is the persistent step
    monkeypatch.delenv("L3_DECODE_PERSIST_MAX_CUS")
    m2 = llama3.Llama(path, args)
    np.testing.assert_array_equal(m2.generate_all(prompt, n), want)
    assert m2.context.decode_persistent()


# (fault position, workgroup that gives up, late): a layer workgroup at the step's start — no
# stage completes, the step writes no cache slot — or an lm workgroup — the layers complete and
# the step writes its K / V slots before the launch fails, so an undo must restore them — or
# (late) a layer workgroup at its last wait of the step: every other layer workgroup writes its
# slots and this one does not, so an undo must restore exactly the others' units (their write
# marks carry the failing launch's tag, decode_persist.hip / kv_restore_kernel)
FAULTS = [(30, 1, 0), (41, 255, 0), (33, 30, 1), (38, 50, 1)]  # wg 30: K units, wg 50: V units


@pytest.mark.parametrize("fault_pos,fault_wg,late", FAULTS)
def test_persistent_decode_fault_recovers_device_loop(tmpdir_mod, monkeypatch, fault_pos, fault_wg, late):
    """One workgroup gives up in the step at fault_pos (L3_DECODE_PERSIST_FAULT, inside an 8-step
    graph of the device loop): every later launch of the graph returns at once; the loop
    recovers — clears the failure words, turns the context graph-only — and runs the rest from
    the failed position on the 25-kernel graph.  145 / 145 ids and every step's value equal the
    reference's, no exception, and the context is graph-only afterwards."""
    g, args, path = _stories(tmpdir_mod, "sharp")
    prompt, want, n = _dream(g)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    monkeypatch.setenv("L3_TEST_FAULT_INJECTION", "1")
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT", str(fault_pos))
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT_WG", str(fault_wg))
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT_LATE", str(late))
    m = llama3.Llama(path, args)
    ids, vals = m.context.greedy_generate(prompt, n, values=True)
    np.testing.assert_array_equal(ids, want)
    ref = np.asarray(g["dream_max"]).reshape(1, -1)
    assert (np.abs(vals - ref) <= ATOL + RTOL * np.abs(ref)).all()
    assert m.context.decode_recoveries() == 1
    assert not m.context.decode_persistent()
    # the context stays correct (graph path) for the next calls
    np.testing.assert_array_equal(m.generate_all(prompt, n), want)
    np.testing.assert_array_equal(np.concatenate(list(m.generate(prompt, n)), axis=1), want)


@pytest.mark.parametrize("fault_pos,fault_wg,late", FAULTS)
def test_persistent_decode_fault_recovers_lazy(tmpdir_mod, monkeypatch, fault_pos, fault_wg, late):
    """The same fault under the lazy generator with run-ahead (llama3.py:310-321: one step per
    yield, the device up to 16 steps ahead): the step that finds the failure undoes every
    queued step — those before the failed one in full, the failed one if it wrote its slots,
    none after it — and runs eagerly; the generator yields the reference's 145 ids.  Then an
    abandoned generator (run-ahead undone on the graph path) and a full one: the KV caches the
    recovery left behind give the reference's ids again."""
    g, args, path = _stories(tmpdir_mod, "sharp")
    prompt, want, n = _dream(g)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    monkeypatch.setenv("L3_TEST_FAULT_INJECTION", "1")
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT", str(fault_pos))
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT_WG", str(fault_wg))
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT_LATE", str(late))
    m = llama3.Llama(path, args)
    got = np.concatenate(list(m.generate(prompt, n)), axis=1)
    np.testing.assert_array_equal(got, want)
    assert m.context.decode_recoveries() == 1
    assert not m.context.decode_persistent()
    gen = m.generate(prompt, n)
    for _ in range(20):
        next(gen)
    del gen
    np.testing.assert_array_equal(np.concatenate(list(m.generate(prompt, n)), axis=1), want)


@pytest.mark.parametrize("fault_wg,late", [(255, 0), (30, 1)])
def test_persistent_decode_fault_in_abandoned_run_ahead(tmpdir_mod, monkeypatch, fault_wg, late):
    """The fault lands in a step the device ran ahead: the consumer stops before it (an
    abandoned generator).  The next call's undo of the abandoned run-ahead (spec_resolve) is
    queued without waiting and decides on the device what to restore (KvGuard): only the slots
    the steps that ran wrote — for the failed step, only its workgroups that wrote (late: all
    but workgroup 30) — and the next decode entry point finishes the recovery (persist_settle);
    the following full generation is exact."""
    g, args, path = _stories(tmpdir_mod, "sharp")
    prompt, want, n = _dream(g)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    monkeypatch.setenv("L3_TEST_FAULT_INJECTION", "1")
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT", "20")
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT_WG", str(fault_wg))
    monkeypatch.setenv("L3_DECODE_PERSIST_FAULT_LATE", str(late))
    m = llama3.Llama(path, args)
    gen = m.generate(prompt, n)
    first = [next(gen) for _ in range(10)]  # positions 5..14 handed out; 15.. queued ahead
    np.testing.assert_array_equal(np.concatenate(first, axis=1), want[:, :10])
    del gen
    np.testing.assert_array_equal(np.concatenate(list(m.generate(prompt, n)), axis=1), want)
    assert m.context.decode_recoveries() == 1


def test_persistent_decode_hd64_instance(tmpdir_mod, monkeypatch):
    """Head dim 64 with D <= 320 and FD in (192, 768] (D 256 = 4 heads of 64, GQA n_rep 2): the
    (D, FD) chunking of stories15M but more old-key dims than its instance holds (KPF 12 = 48
    dims) — the instance table picks KPF 16.  Greedy ids of the persistent step (device loop and
    lazy) equal the oracle's and the 25-kernel graph's."""
    args = ModelArgs(dim=256, n_layers=2, n_heads=4, n_kv_heads=2, vocab_size=512, max_seq_len=96,
                     max_batch_size=1)
    w = synth.make_weights(args, 512, seed=7, preset="sharp")
    path = os.path.join(tmpdir_mod, "hd64.npz")
    synth.save_npz(path, w)
    prompt = np.random.default_rng(3).integers(0, args.vocab_size, (1, 7))
    n = 80
    want = orc.greedy_ids(orc.OracleModel(w, args), prompt, n)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    m = llama3.Llama(path, args)
    np.testing.assert_array_equal(m.generate_all(prompt, n), want)
    assert m.context.decode_persistent()
    np.testing.assert_array_equal(np.concatenate(list(m.generate(prompt, n)), axis=1), want)
    monkeypatch.setenv("L3_DECODE_PERSIST", "0")
    m0 = llama3.Llama(path, args)
    np.testing.assert_array_equal(m0.generate_all(prompt, n), want)
    assert not m0.context.decode_persistent()


# (dim, heads, kv heads, hidden, seed) -> the persistent step's instances by their (D, FD)
# chunking (decode_persist.hip L3_PERSIST_INSTANCES): (1, 12), (5, 3), (5, 16), (8, 16), (8, 12);
# the seeds' smallest top-2 margins over the run are 0.023 / 0.023 / 0.055 / 0.035 / 0.071
INSTANCE_SHAPES = [(64, 1, 1, 512, 32), (128, 2, 2, 128, 33), (256, 4, 4, 1024, 32), (512, 8, 4, 1024, 32),
                   (384, 8, 8, 768, 31)]


@pytest.mark.parametrize("dim,heads,kv_heads,hidden,seed", INSTANCE_SHAPES)
def test_persistent_decode_instances(tmpdir_mod, monkeypatch, dim, heads, kv_heads, hidden, seed):
    """Every persistent-step instance the stories15M / tiny tests do not reach: 91 greedy steps
    (max_seq_len 96) on the persistent step, ids and winning logits against the oracle."""
    args = ModelArgs(dim=dim, n_layers=2, n_heads=heads, n_kv_heads=kv_heads, vocab_size=512, max_seq_len=96,
                     max_batch_size=1)
    w = synth.make_weights(args, hidden, seed=seed, preset="sharp")
    path = os.path.join(tmpdir_mod, f"inst{dim}_{hidden}.npz")
    synth.save_npz(path, w)
    prompt = np.random.default_rng(seed).integers(0, args.vocab_size, (1, 5))
    n = args.max_seq_len
    want, wv = _oracle_greedy_values(orc.OracleModel(w, args), prompt, n)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    m = llama3.Llama(path, args)
    ids, vals = m.context.greedy_generate(prompt, n, values=True)
    assert m.context.decode_persistent()
    np.testing.assert_array_equal(ids, want)
    err = np.abs(vals.astype(np.float64) - wv)
    assert (err <= ATOL + RTOL * np.abs(wv)).all(), f"worst step {int(err.argmax())}: {err.max():.3e}"


def test_persistent_decode_past_256_keys(tmpdir_mod, monkeypatch):
    """Contexts longer than the persistent step's 256-thread workgroup (max_seq_len 700): the
    attention stage's second-pass loops (scores of keys past the first 256 and their P.V rows
    read from the cache) run for every step past position 256.  A 693-step greedy run from a
    7-token prompt — ids and each step's winning logit against the oracle (smallest top-2
    margin of this run 6.9e-3, |logits| <= 12.7) — on the persistent step in the device loop
    and the lazy generator, and on the 25-kernel graph."""
    args = ModelArgs(dim=64, n_layers=2, n_heads=2, n_kv_heads=1, vocab_size=512, max_seq_len=700,
                     max_batch_size=1)
    w = synth.make_weights(args, 128, seed=22, preset="sharp")
    path = os.path.join(tmpdir_mod, "long.npz")
    synth.save_npz(path, w)
    prompt = np.random.default_rng(5).integers(0, args.vocab_size, (1, 7))
    n = args.max_seq_len
    want, wv = _oracle_greedy_values(orc.OracleModel(w, args), prompt, n)
    monkeypatch.setenv("L3_DECODE_PERSIST", "1")
    m = llama3.Llama(path, args)
    ids, vals = m.context.greedy_generate(prompt, n, values=True)
    assert m.context.decode_persistent()
    np.testing.assert_array_equal(ids, want)
    err = np.abs(vals.astype(np.float64) - wv)
    assert (err <= ATOL + RTOL * np.abs(wv)).all(), f"worst step {int(err.argmax())}: {err.max():.3e}"
    np.testing.assert_array_equal(np.concatenate(list(m.generate(prompt, n)), axis=1), want)
    assert m.context.decode_recoveries() == 0
    monkeypatch.setenv("L3_DECODE_PERSIST", "0")
    m0 = llama3.Llama(path, args)
    np.testing.assert_array_equal(m0.generate_all(prompt, n), want)
    assert not m0.context.decode_persistent()
    print(f"693 steps past 256 keys: ids exact, values max-abs {err.max():.2e}")


def _oracle_greedy_values(ref, prompt, max_new):
    """The reference's greedy loop (llama3.py:310-321) on the oracle, with each step's winning
    logit (the value np.argmax picked at :320)."""
    ids, vals, nxt = [], [], None
    L = prompt.shape[1]
    for i, pos in enumerate(range(L, max_new)):
        logits = ref(prompt, 0) if i == 0 else ref(nxt, pos)
        last = logits[:, -1, :]
        nxt = last.argmax(-1)[:, None]
        ids.append(nxt)
        vals.append(last.max(-1)[:, None])
    return np.concatenate(ids, axis=1), np.concatenate(vals, axis=1)


@pytest.mark.parametrize("B", [9, 16, 64, 256])
def test_batched_decode_lm_head_partials(tmpdir_mod, B):
    """Batched device loop (B > 8: the tiled lm_head, whose captured steps leave per-row argmax
    partials instead of the logits, GemmArgs::amax_rows, reduced in one B-row launch): the ids
    and each step's winning logit of three spread rows equal the oracle's (rows never interact,
    llama3.py:163-211), every row's ids equal a second run's."""
    args = synth.stories15m(B)
    path = os.path.join(tmpdir_mod, f"b{B}.npz")
    w = synth.make_weights(args, synth.STORIES15M_HIDDEN, seed=11, preset="sharp")
    synth.save_npz(path, w)
    prompt = np.random.default_rng(B).integers(0, args.vocab_size, (B, 5))
    n = 30
    m = llama3.Llama(path, args)
    ids, vals = m.context.greedy_generate(prompt, n, values=True)
    for r in (0, B // 2, B - 1):
        ref = orc.OracleModel(w, synth.stories15m(1))
        want, wv = _oracle_greedy_values(ref, prompt[r:r + 1], n)
        np.testing.assert_array_equal(ids[r:r + 1], want, err_msg=f"row {r}")
        assert (np.abs(vals[r:r + 1] - wv) <= ATOL + RTOL * np.abs(wv)).all(), f"row {r}"
    np.testing.assert_array_equal(llama3.Llama(path, args).generate_all(prompt, n), ids)
