"""CPU checks of the x6 GEMM path's arithmetic (llama3.np_amd/csrc/gemm_x6.h): the three-piece
bf16 cut is exact, and the six kept piece products carry an fp32 dot product to fp32 accuracy.

The kernel cuts x by truncation: hi = x with the low 16 bits cleared, r = x - hi, mid = r with the
low 16 bits cleared, lo = r - mid (split3_one); every piece is a bf16 (low half zero) and
x = hi + mid + lo exactly.  The MFMA forms each bf16 x bf16 product exactly and accumulates in
fp32; six products are kept (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid).
"""
import numpy as np


def split3(x):
    """NumPy restatement of gemm_x6.h split3_one (fp32 in, three fp32 arrays holding bf16s)."""
    x = np.asarray(x, np.float32)
    hi = (x.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32)
    r = (x - hi).astype(np.float32)
    mid = (r.view(np.uint32) & np.uint32(0xFFFF0000)).view(np.float32)
    lo = (r - mid).astype(np.float32)
    return hi, mid, lo


def _rand_f32(rng, n):
    # random signs, significands and exponents across the normal range the model produces
    m = rng.uniform(1.0, 2.0, n)
    e = rng.integers(-40, 40, n)
    return (np.sign(rng.standard_normal(n)) * m * np.exp2(e)).astype(np.float32)


def test_split_is_exact_and_pieces_are_bf16():
    rng = np.random.default_rng(0)
    x = np.concatenate([_rand_f32(rng, 1_000_000), np.float32([0.0, -0.0, 1.0, -1.0, 3.0e-30, 6.5e4]),
                        rng.standard_normal(100_000).astype(np.float32)])
    hi, mid, lo = split3(x)
    for piece in (hi, mid, lo):
        assert not (piece.view(np.uint32) & np.uint32(0xFFFF)).any()  # a bf16 in the top half
    # exact: the sum in float64 reproduces x bit for bit
    np.testing.assert_array_equal((hi.astype(np.float64) + mid + lo).astype(np.float32), x)
    assert np.array_equal(hi.astype(np.float64) + mid + lo, x.astype(np.float64))
    # the pieces' sizes behind the dropped-term bound: |mid| < 2^-7 |x|, |lo| < 2^-15 |x|
    nz = x != 0
    assert (np.abs(mid[nz]) < np.abs(x[nz]) * 2.0 ** -7).all()
    assert (np.abs(lo[nz]) < np.abs(x[nz]) * 2.0 ** -15).all()


def _dot_x6(a, w):
    """The kernel's arithmetic for an output block: per 32-deep k step, six
    v_mfma_f32_16x16x32_bf16 (the kernel's order: mid.mid, lo.hi, hi.lo, mid.hi, hi.mid, hi.hi),
    each modelled as its 32 exact bf16 x bf16 products summed and added to the fp32 accumulator
    with one rounding (the measured hardware error is in tools/gemm_tune x6acc)."""
    ah, am, al = split3(a)
    wh, wm, wl = split3(w)
    acc = np.zeros((a.shape[0], w.shape[0]), np.float32)
    for k0 in range(0, a.shape[1], 32):
        ks = slice(k0, k0 + 32)
        for x, y in ((am, wm), (ah, wl), (al, wh), (ah, wm), (am, wh), (ah, wh)):
            p = x[:, ks].astype(np.float64) @ y[:, ks].astype(np.float64).T
            acc = (acc.astype(np.float64) + p).astype(np.float32)
    return acc


def _dot_fp32(a, w):
    """The fp32 kernel's: v_mfma_f32_16x16x4_f32 is an fmaf chain (MI355X_MICROARCH.md), one
    rounding per k."""
    acc = np.zeros((a.shape[0], w.shape[0]), np.float32)
    for k in range(a.shape[1]):
        acc = (acc.astype(np.float64) + a[:, k:k + 1].astype(np.float64) * w[:, k].astype(np.float64)[None, :]).astype(np.float32)
    return acc


def test_six_products_reach_fp32_accuracy():
    """Against the float64 product, the six-product sum's error is at or below the fp32 kernel's
    (an fmaf chain over k): the dropped mid.lo, lo.mid, lo.lo terms sit under fp32's rounding of
    each product, and six roundings per 32 k replace 32 (both as modelled above)."""
    rng = np.random.default_rng(1)
    a = rng.uniform(-1, 1, (64, 288)).astype(np.float32)
    w = rng.uniform(-0.05, 0.05, (48, 288)).astype(np.float32)
    ref = a.astype(np.float64) @ w.astype(np.float64).T
    e6 = np.abs(_dot_x6(a, w) - ref)
    e32 = np.abs(_dot_fp32(a, w) - ref)
    assert e6.max() <= e32.max()
    assert np.sqrt((e6 ** 2).mean()) <= np.sqrt((e32 ** 2).mean())
    # and the dropped terms alone are an order of magnitude below either (measured 0.08x here):
    # the exact six-term sum vs the full product
    ah, am, al = split3(a)
    wh, wm, wl = split3(w)
    six = sum(x.astype(np.float64) @ y.astype(np.float64).T
              for x, y in ((am, wm), (ah, wl), (al, wh), (ah, wm), (am, wh), (ah, wh)))
    assert np.abs(six - ref).max() < 0.15 * e32.max()
