"""CPU: the oracle's two fp16 V-accumulator steps (oracle/qasr_oracle.c
qo_f16_mad_round2 = ggml_vec_mad_f16 on F16C, fp16(fmaf(x, v, y)); and
qo_f16_mad_round1 = the single-rounding variant of QO_FA_V_ROUND1) against
exact rational arithmetic: round1 is RNE-to-fp16 of the exact x * v + y,
round2 is RNE-to-fp16 of RNE-to-fp32 of it.  Random triples plus constructed
cases whose fp32 rounding lands on an fp16 midpoint (where the two differ)."""
from fractions import Fraction

import numpy as np

import oracle_py as op


def _rne_int(m: Fraction) -> int:
    n = m.numerator // m.denominator
    r = m - n
    if r > Fraction(1, 2) or (r == Fraction(1, 2) and n & 1):
        n += 1
    return n


def _binade(a: Fraction) -> int:
    """e with 2^e <= a < 2^(e+1), a > 0"""
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    elif Fraction(2) ** (e + 1) <= a:
        e += 1
    return e


def f16_rne(q: Fraction) -> int:
    """bits of RNE-to-fp16(q), q exact"""
    sign = 0x8000 if q < 0 else 0
    a = abs(q)
    if a == 0:
        return sign
    if a >= 65520:
        return sign | 0x7C00
    ue = max(_binade(a) - 10, -24)
    n = _rne_int(a / Fraction(2) ** ue)
    if n < 1024:   # subnormal (ue == -24)
        return sign | n
    E = ue + 25
    if n == 2048:
        E, n = E + 1, 1024
    return sign | 0x7C00 if E >= 31 else sign | (E << 10) | (n - 1024)


def f32_rne(q: Fraction) -> Fraction:
    """RNE-to-fp32(q) as an exact value (fp16 range only: no fp32 overflow)"""
    if q == 0:
        return Fraction(0)
    a = abs(q)
    ue = max(_binade(a) - 23, -149)
    v = _rne_int(a / Fraction(2) ** ue) * Fraction(2) ** ue
    return v if q > 0 else -v


def _h(bits: int) -> Fraction:
    return Fraction(float(np.array([bits], np.uint16).view(np.float16)[0]))


def _cases(n_rand: int = 4000):
    rng = np.random.default_rng(7)
    out = []
    for _ in range(n_rand):
        xb = int(rng.integers(0, 0x7C00)) | (0x8000 if rng.random() < 0.3 else 0)
        yb = int(rng.integers(0, 0x7C00)) | (0x8000 if rng.random() < 0.3 else 0)
        kind = rng.integers(0, 3)
        v = float(np.float32(rng.random() if kind == 0 else np.exp(-rng.random() * 30) if kind == 1 else rng.random() * 1e-6))
        out.append((xb, v, yb))
    # constructed: y = 1.0, x * v = half an fp16 ulp of 1 plus a tail below fp32's ulp
    # (fp32 rounds onto the midpoint, the exact value is above or below it)
    one = 0x3C00
    for t in (2.0 ** -34, -(2.0 ** -34), 2.0 ** -33, 2.0 ** -40):
        out.append((one, float(np.float32(2.0 ** -11 + t)), one))
    # the same across binades and signs, and in the fp16 subnormal range
    for e in range(-14, 15, 3):
        yb = int(np.array([2.0 ** e], np.float16).view(np.uint16)[0])
        out.append((one, float(np.float32(2.0 ** (e - 11) * (1 + 2.0 ** -23))), yb))
        out.append((one | 0x8000, float(np.float32(2.0 ** (e - 11) * (1 + 2.0 ** -23))), yb | 0x8000))
    out.append((0x0001, float(np.float32(0.5 + 2.0 ** -24)), 0x0002))   # subnormal tie region
    out.append((0x0001, 0.5, 0x0002))                                   # an exact tie (to even)
    return out


def test_mad_round1_is_exact_rne(built):
    L = op.olib()
    n_diff = 0
    for xb, v, yb in _cases():
        exact = _h(xb) * Fraction(v) + _h(yb)
        r1 = L.qo_f16_mad_round1(xb, v, yb)
        r2 = L.qo_f16_mad_round2(xb, v, yb)
        assert r1 == f16_rne(exact), (hex(xb), v, hex(yb), hex(r1), hex(f16_rne(exact)))
        assert r2 == f16_rne(f32_rne(exact)), (hex(xb), v, hex(yb), hex(r2))
        n_diff += r1 != r2
    assert n_diff >= 4   # the constructed double-rounding cases do differ
