"""Generate the committed golden fixtures by running the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only; nothing is
copied from it — only its outputs on synthetic inputs are saved):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --c5   # Llama-3-shape slice

The reference ships no golden vectors, so these fixtures are
the parity anchor: the oracle (oracle/llama3_oracle.py) is pinned against them
in tests/test_oracle_golden.py, and the GPU path is checked against both.

Weights are synthetic (llama3.np_amd/synth.py, fixed seeds) because
stories15M.model.npz is absent offline; their sha256 is recorded so a drift in
the generator is caught.
"""

import json
import os
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
import synth  # noqa: E402  (product-side generator; numpy only)

# the product's modules share the reference's module names: drop them so the
# imports below bind the reference's own config/llama3/tokenizer
sys.path.pop(0)
for _m in ("config", "tokenizer", "utils", "llama3"):
    sys.modules.pop(_m, None)
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import config as ref_config  # noqa: E402
import llama3 as ref  # noqa: E402
import tokenizer as ref_tok  # noqa: E402


def ref_args(args):
    """Same field values, but the reference's own ModelArgs class."""
    return ref_config.ModelArgs(**{k: getattr(args, k) for k in args.__dataclass_fields__})


def tokenizer_fixture():
    tok = ref_tok.Tokenizer(os.path.join(REF, "tokenizer.model.np"))
    prompts = ["I have a dream", "Once upon a time", "", "a", "Hello, world!",
               "The quick brown fox jumps over the lazy dog.",
               "Lily and Ben were playing in the park. They saw a big red ball!",
               "tab\tnew\nline  double  space", "ümlaut café 你好 ☃",
               "<s> tags </s> inside"]
    enc = []
    for p in prompts:
        enc.append({"text": p, "ids": tok.encode(p),
                    "ids_eos": tok.encode(p, add_bos=False, add_eos=True)})
    rng = np.random.default_rng(7)
    id_lists = [[471], [29879], [1, 76, 505, 263, 12561], [2], [1], [0], [3, 4, 13],
                [26222, 2501, 263, 931]] + [rng.integers(0, 32000, 6).tolist() for _ in range(8)]
    dec = [{"ids": ids, "text": tok.decode(ids)} for ids in id_lists]
    with open(os.path.join(HERE, "tokenizer.json"), "w", encoding="utf-8") as f:
        json.dump({"encode": enc, "decode": dec}, f, ensure_ascii=False, indent=0)


def ops_fixture():
    rng = np.random.default_rng(11)
    out = {}
    x = rng.standard_normal((2, 6, 8, 8)).astype(np.float32)
    out["softmax_x"], out["softmax_y"] = x, ref.softmax(x)
    xm = x.astype(np.float64) + np.triu(np.full((8, 8), -np.inf), 1)
    out["softmax_masked_x"], out["softmax_masked_y"] = xm, ref.softmax(xm)
    x = rng.standard_normal((2, 8, 288)).astype(np.float32) * 3
    out["silu_x"], out["silu_y"] = x, ref.silu(x)
    c, s = ref.compute_cos_sin_cache(48, 256)
    out["rope_cos"], out["rope_sin"] = c, s
    xq = rng.standard_normal((2, 8, 6, 48)).astype(np.float32)
    xk = rng.standard_normal((2, 8, 2, 48)).astype(np.float32)
    oq, ok = ref.apply_rotary_emb(xq, xk, c[3:11], s[3:11])
    out.update(rope_xq=xq, rope_xk=xk, rope_start=np.int64(3), rope_q=oq, rope_k=ok)
    x = rng.standard_normal((2, 8, 288)).astype(np.float32)
    w = rng.standard_normal(288).astype(np.float32)
    out.update(rms_x=x, rms_w=w, rms_y=ref.RMSNorm(w, 1e-6)(x))
    x64 = x.astype(np.float64)
    out.update(rms64_x=x64, rms64_y=ref.RMSNorm(w, 1e-6)(x64))
    xf = rng.standard_normal((2, 8, 64)).astype(np.float32)
    wg = (rng.standard_normal((192, 64)) * 0.2).astype(np.float32)
    wu = (rng.standard_normal((192, 64)) * 0.2).astype(np.float32)
    wd = (rng.standard_normal((64, 192)) * 0.2).astype(np.float32)
    ff = ref.FeedForward(wu, wg, wd)
    out.update(ffn_x=xf, ffn_wg=wg, ffn_wu=wu, ffn_wd=wd, ffn_y=ff(xf))
    kv = rng.standard_normal((1, 5, 2, 4))
    out.update(repkv_x=kv, repkv_y=ref.repeat_kv(kv, 3))
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **out)


def model_fixture(tmp, name, args, hidden, seed, preset, cases, gen=None):
    w = synth.make_weights(args, hidden, seed=seed, preset=preset)
    path = os.path.join(tmp, name + ".npz")
    synth.save_npz(path, w)
    out = {"weights_sha256": np.array(synth.digest(w)), "seed": np.int64(seed),
           "preset": np.array(preset)}
    model = ref.Llama(path, ref_args(args))
    # sequential calls on ONE model: caches persist, exactly like the reference
    for tag, ids, start in cases:
        out[f"{tag}_ids"] = ids
        out[f"{tag}_start"] = np.int64(start)
        out[f"{tag}_logits"] = model(ids, start)
    if gen is not None:
        gtag, gids, max_new = gen
        gm = ref.Llama(path, ref_args(args))
        steps, margins, maxes = [], [], []
        # replicate Llama.generate but also record the top-2 margin and the winning logit of
        # each step
        L = gids.shape[1]
        nxt = None
        for i, pos in enumerate(range(L, max_new)):
            logits = gm(gids, 0) if i == 0 else gm(nxt, pos)
            srt = np.sort(logits[:, -1, :], axis=-1)
            margins.append(srt[:, -1] - srt[:, -2])
            maxes.append(srt[:, -1])
            nxt = logits[:, -1, :].argmax(-1, keepdims=True)
            steps.append(nxt)
        ids_ref = np.concatenate(list(ref.Llama(path, ref_args(args)).generate(gids, max_new)), axis=1)
        got = np.concatenate(steps, axis=1)
        assert np.array_equal(ids_ref, got)
        out[f"{gtag}_prompt"] = gids
        out[f"{gtag}_max_new"] = np.int64(max_new)
        out[f"{gtag}_ids"] = got
        out[f"{gtag}_margin"] = np.stack(margins, axis=1)
        out[f"{gtag}_max"] = np.stack(maxes, axis=1)  # the logit np.argmax picked, per step
        # decode hole: layer-0 cache rows that are still exactly zero after generate
        ck = gm.layers[0].attention.cache_k
        out[f"{gtag}_zero_slots"] = np.nonzero(np.all(ck[0] == 0, axis=(1, 2)))[0][:8]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return out


def c5_slice_fixture(tmp):
    """a 2-layer Llama-3-8B-shaped slice (D 4096, H 32 / KVH 8, HD 128,
    FD 14336, VS 128256), B = 1: prefill L = 256, then two decode steps at the reference's
    positions (257, 258: slot 256 is the decode hole).  Only ids and logits are stored; the
    6 GB weight set is regenerated from the seed (its sha256 is recorded)."""
    args = synth.llama3_shape(n_layers=2, max_batch_size=1)
    rng = np.random.default_rng(5)
    ids = rng.integers(0, args.vocab_size, (1, 256))
    d1 = rng.integers(0, args.vocab_size, (1, 1))
    d2 = rng.integers(0, args.vocab_size, (1, 1))
    model_fixture(tmp, "c5_slice", args, synth.LLAMA3_HIDDEN, 2, "default",
                  [("prefill", ids, 0), ("dec1", d1, 257), ("dec2", d2, 258)])


def main():
    if "--c5" in sys.argv:  # separate: ~6 GB of weights, about a minute of reference CPU time
        with tempfile.TemporaryDirectory(dir=os.environ.get("GOLDEN_TMP")) as tmp:
            c5_slice_fixture(tmp)
        print("c5 fixture written to", HERE)
        return
    tokenizer_fixture()
    ops_fixture()
    rng = np.random.default_rng(3)
    with tempfile.TemporaryDirectory() as tmp:
        # tiny model with GQA (n_rep = 2): prefill, chunked prefill at start_pos>0, decode
        t = synth.tiny(max_batch_size=4)
        ids_a = rng.integers(0, t.vocab_size, (4, 12))
        ids_b = rng.integers(0, t.vocab_size, (4, 5))
        ids_c = rng.integers(0, t.vocab_size, (4, 1))
        model_fixture(tmp, "tiny", t, synth.TINY_HIDDEN, 5, "sharp",
                      [("prefill", ids_a, 0), ("chunk", ids_b, 12), ("decode", ids_c, 18)],
                      gen=("gen", rng.integers(0, t.vocab_size, (2, 6)), 40))
        # stories15M shape, both presets; greedy "I have a dream" = [1,76,505,263,12561]
        s = synth.stories15m(max_batch_size=2)
        prompt = np.array([[1, 76, 505, 263, 12561]])
        ids = rng.integers(0, s.vocab_size, (2, 16))
        for preset, seed in (("default", 0), ("sharp", 1)):
            model_fixture(tmp, f"stories15m_{preset}", s, synth.STORIES15M_HIDDEN, seed, preset,
                          [("prefill", ids, 0)], gen=("dream", prompt, 150))
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
