"""The bf16 mode's fused FeedforwardModule alone, against a float64 product of the same bf16
operands (zasr_selftest_ffn_bf16).

ffn_fused_kernel (d <= 192), ffn_wide_kernel (d = 256..512) and the opt-in per-CU rows form
ffn_rows_kernel (d = 384, form 1: 64-token tiles and a 16-48-token tail tile per block) over the row
counts the decode meets only incidentally: M < 16, one 16-row group either side of a 64-token
tile, per-CU shares of 1-2 tiles with every tail length (rpb = 32, 64, 80, 112, 128 at 256
CUs) and a ragged last block.  The reference rounds X, W1, W2 and the hidden activation to
bf16 exactly as the kernels do (round to nearest even), so what remains is f32 accumulation
order and the odd hidden value whose bf16 rounding flips: max |got - ref| <= 2e-3 of the
FFN output's max |.| (measured ~1e-4, tools/ffnw_lab.hip).
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

BOUND = 2e-3


@pytest.fixture(scope="module")
def need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")


def bf16(x):
    """float32 -> bf16 (round to nearest even) -> float64, as (__bf16)x on the device."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return (r & 0xFFFFFFFF).astype(np.uint32).view(np.float32).astype(np.float64)


def _swooshl(x):
    return np.logaddexp(0.0, x - 4.0) - 0.08 * x - 0.035


FFN_CASES = [(128, 384, False, 0), (192, 512, False, 0), (192, 640, True, 0), (256, 768, False, 0),
             (384, 1024, False, 0), (384, 1024, False, 1), (384, 1280, True, 1), (512, 1536, False, 0)]
ROWS = (1, 15, 17, 63, 65, 256 * 16 + 7, 256 * 48 + 5)
# d = 384 (the rows form): shares of 80 / 112 / 128 rows (a tile + a 1-group / 3-group tail,
# two tiles), the last block ragged
ROWS_384 = ROWS + (256 * 70 + 3, 256 * 100 + 9, 256 * 112 + 5)


@pytest.mark.parametrize("D,F,byp,form", FFN_CASES,
                         ids=[f"D{d}_F{f}{'_byp' if b else ''}{'_rows' if r else ''}"
                              for d, f, b, r in FFN_CASES])
def test_ffn_bf16_matches_f64(need_gpu, D, F, byp, form):
    from zasr.binding import selftest_ffn_bf16
    rng = np.random.default_rng(9100 + D + F + byp + 7 * form)
    W1 = (rng.standard_normal((F, D)) / np.sqrt(D)).astype(np.float32)
    W2 = (rng.standard_normal((D, F)) / np.sqrt(F)).astype(np.float32)
    b1 = rng.standard_normal(F).astype(np.float32) * 0.5
    b2 = rng.standard_normal(D).astype(np.float32) * 0.1
    ks = rng.uniform(0.3, 0.9, D).astype(np.float32)
    w1, w2 = bf16(W1), bf16(W2)
    worst = 0.0
    for R in (ROWS_384 if form == 1 else ROWS):
        X = rng.standard_normal((R, D)).astype(np.float32)
        bo = rng.standard_normal((R, D)).astype(np.float32) if byp else None
        got = selftest_ffn_bf16(W1, b1, W2, b2, X, bo, ks if byp else None, form=form)
        h = bf16(_swooshl(bf16(X) @ w1.T + b1.astype(np.float64)).astype(np.float32))
        o = h @ w2.T + b2.astype(np.float64)
        ref = X.astype(np.float64) + o
        if byp:
            ref = bo + (ref - bo) * ks.astype(np.float64)
        e = float(np.max(np.abs(got.astype(np.float64) - ref)) / np.max(np.abs(o)))
        worst = max(worst, e)
        assert e <= BOUND, (D, F, R, byp, e)
    print(f"D={D} F={F} byp={byp} form={form}: worst {worst:.2e}")
