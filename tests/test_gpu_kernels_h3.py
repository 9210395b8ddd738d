"""The f16x3 one-accumulator kernels alone, against a float64 product.

gemm_h3r_kernel (row-resident projection GEMM) and ffn_wide_h3_kernel (fused FeedforwardModule)
run through zasr_selftest_gemm_h3r / zasr_selftest_ffn_h3 on seeded host operands, over every
K / D and epilogue the engine routes to them and the row counts the decode meets only
incidentally: M = 1, 15, 17, one 16-row group either side of the tile height (16 TUM +- 1), a
per-CU share with a partial tail (256 * 16 + 7 rows: every block one 32-row share, the last
one ragged) and a multi-tile share.  Bound: the f16x3 format carries 22 significand bits per
operand (hi + lo 2^-11 pieces, products accumulated in f32), so the output's error is a few
f32 ulps of its scale -- max |got - ref| <= 3e-6 * max |ref| (measured <= 1.9e-6) (the SwooshL / sigmoid epilogues
use native exp2 / log2 / rcp, ~1e-7 relative).
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

BOUND = 3e-6
EPI_NONE, EPI_RESADD, EPI_GLU = 0, 3, 8


@pytest.fixture(scope="module")
def need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")


def h3r_tile_groups(K, epi):
    """gemm_h3r.hip: 16-row groups per tile (the LDS bound and the VGPR cap)."""
    xld = K + (16 if K % 64 == 0 else 48)
    tul = 160 * 1024 // (64 * xld)
    tumx = 8 if K <= 192 else (6 if (K <= 256 or (K <= 384 and epi != EPI_RESADD)) else 4)
    return min(tul, tumx)


def rows_sweep(tum):
    return sorted({1, 15, 17, 16 * tum - 1, 16 * tum + 1, 256 * 16 + 7, 256 * 16 * 3 + 5})


def _rel_err(got, ref):
    return float(np.max(np.abs(got.astype(np.float64) - ref)) / max(1e-30, np.max(np.abs(ref))))


H3R_CASES = [(K, epi) for K in (96, 192, 256, 288, 384, 512) for epi in (EPI_NONE, EPI_RESADD, EPI_GLU)
             if epi == EPI_NONE or K >= 256]


@pytest.mark.parametrize("K,epi", H3R_CASES, ids=[f"K{k}_epi{e}" for k, e in H3R_CASES])
def test_gemm_h3r_matches_f64(need_gpu, K, epi):
    from zasr.binding import selftest_gemm_h3r
    rng = np.random.default_rng(1000 + K + epi)
    worst = 0.0
    for N in (128, 272):
        W = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)
        W[0, 0] = 30.5  # the largest magnitude the one-accumulator form takes (< 31)
        b = rng.standard_normal(N).astype(np.float32) * 0.1
        for M in rows_sweep(h3r_tile_groups(K, epi)):
            A = rng.standard_normal((M, K)).astype(np.float32)
            ncol = N // 2 if epi == EPI_GLU else N
            C0 = rng.standard_normal((M, ncol)).astype(np.float32)
            got = selftest_gemm_h3r(A, W, b, C0, epi)
            v = A.astype(np.float64) @ W.astype(np.float64).T + b.astype(np.float64)
            if epi == EPI_RESADD:
                ref = C0.astype(np.float64) + v
            elif epi == EPI_GLU:
                ref = v[:, 0::2] / (1.0 + np.exp(-v[:, 1::2]))
            else:
                ref = v
            e = _rel_err(got, ref)
            worst = max(worst, e)
            assert e <= BOUND, (K, N, M, epi, e)
    print(f"K={K} epi={epi}: worst {worst:.2e}")


def test_gemm_h3r_refuses_out_of_range_weights(need_gpu):
    """|w| >= 31 leaves the one-accumulator kernel's exact range: the self-test refuses it, as
    the engine routes such a layer to gemm_x3 (tests/test_gpu_routes.py)."""
    from zasr.binding import ZasrError, selftest_gemm_h3r
    A = np.ones((16, 256), np.float32)
    W = np.zeros((128, 256), np.float32)
    W[5, 7] = 31.0
    with pytest.raises(ZasrError, match="31"):
        selftest_gemm_h3r(A, W, None, np.zeros((16, 128), np.float32))


def _swooshl(x):
    return np.logaddexp(0.0, x - 4.0) - 0.08 * x - 0.035


FFN_CASES = [(128, 384, 8, False), (192, 512, 4, False), (192, 640, 4, True), (256, 768, 5, False),
             (384, 1024, 4, True), (384, 1024, 4, False), (512, 1536, 3, False)]


@pytest.mark.parametrize("D,F,tum,byp", FFN_CASES, ids=[f"D{d}_F{f}{'_byp' if b else ''}"
                                                        for d, f, _, b in FFN_CASES])
def test_ffn_h3_matches_f64(need_gpu, D, F, tum, byp):
    from zasr.binding import selftest_ffn_h3
    rng = np.random.default_rng(7000 + D + F + byp)
    W1 = (rng.standard_normal((F, D)) / np.sqrt(D)).astype(np.float32)
    W2 = (rng.standard_normal((D, F)) / np.sqrt(F)).astype(np.float32)
    W1[3, 1] = -30.5
    b1 = rng.standard_normal(F).astype(np.float32) * 0.5
    b2 = rng.standard_normal(D).astype(np.float32) * 0.1
    ks = rng.uniform(0.3, 0.9, D).astype(np.float32)
    worst = 0.0
    for R in rows_sweep(tum):
        if R > 20000 and D >= 384:
            R = 256 * 16 * 2 + 3  # keep the f64 reference product bounded
        Y = rng.standard_normal((R, D)).astype(np.float32)
        X = rng.standard_normal((R, D)).astype(np.float32)
        bo = rng.standard_normal((R, D)).astype(np.float32) if byp else None
        got = selftest_ffn_h3(Y, W1, b1, W2, b2, X, bo, ks if byp else None)
        h = _swooshl(Y.astype(np.float64) @ W1.astype(np.float64).T + b1)
        ref = X.astype(np.float64) + h @ W2.astype(np.float64).T + b2
        if byp:
            ref = bo + (ref - bo) * ks.astype(np.float64)
        e = _rel_err(got, ref)
        worst = max(worst, e)
        assert e <= BOUND, (D, F, R, byp, e)
    print(f"D={D} F={F} byp={byp}: worst {worst:.2e}")
