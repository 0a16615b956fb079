#!/usr/bin/env python3
"""Fit of the degree-6 exp() polynomial of the split-exponent arithmetic (xf_exp: oracle
EC[], csrc/xf_math.h, csrc/lattice_dev.h xf_exp_pair).

e^r on [-ln2/2, ln2/2] with c0 = c1 = 1 and c2 = 1/2 fixed (exact, and 0.5 stays an inline
constant of v_pk_fma_f32), c3..c6 by iteratively reweighted least squares towards the
relative-error minimax, then rounded to f32. Prints the coefficients, the approximation error
and the statistics of the f32 Horner evaluation (fma emulated in float64) over log-probs.

Why: the previous coefficients' error curve was one-sided (0.33 ulp at
r = -0.3); summed over the ~2000 factors of a configs[4] path that bias alone moved log-alpha
by ~4e-6 and pushed the f32 recurrence past the north_star 1e-5 in 5 of 64 (utterance,
direction) cases. With these coefficients the largest of 64 is 9.6e-6.
"""
import numpy as np

H = np.log(2.0) / 2


def fit():
    r = np.linspace(-H, H, 40001)
    f = np.exp(r)
    A = np.stack([r ** k / f for k in range(3, 7)], 1)
    y = (f - 1 - r - 0.5 * r * r) / f
    w = np.ones_like(r)
    for _ in range(300):
        c, *_ = np.linalg.lstsq(A * np.sqrt(w)[:, None], y * np.sqrt(w), rcond=None)
        res = np.abs(A @ c - y)
        w = w * (res / res.max() + 1e-3) ** 0.3
        w /= w.mean()
    return [1.0, 1.0, 0.5] + [float(np.float32(x)) for x in c]


def approx_err_ulp(C):
    r = np.linspace(-H, H, 20001)
    p = np.zeros_like(r)
    for k in range(6, -1, -1):
        p = p * r + C[k]
    return float(np.abs((p - np.exp(r)) / np.exp(r)).max() / 2.0 ** -24)


def f32_eval_stats(C, n=2_000_000, seed=7):
    rng = np.random.default_rng(seed)
    x = (-rng.random(n) * 12.0).astype(np.float32)
    f32 = np.float32
    L2E, LN2HI, LN2LO = f32(float.fromhex("0x1.715476p+0")), f32(float.fromhex("0x1.62e400p-1")), \
        f32(float.fromhex("0x1.7f7d1cp-20"))
    fma = lambda a, b, c: (a.astype(np.float64) * b + c).astype(np.float32)  # noqa: E731
    nn = np.rint(x * L2E).astype(np.float32)
    r = fma(-nn, LN2HI, x)
    r = fma(-nn, LN2LO, r)
    p = np.full_like(r, f32(C[6]))
    for k in range(5, -1, -1):
        p = fma(p, r, f32(C[k]))
    v = np.ldexp(p.astype(np.float64), nn.astype(np.int64))
    rel = (v - np.exp(x.astype(np.float64))) / np.exp(x.astype(np.float64)) / 2.0 ** -24
    return float(rel.mean()), float(np.sqrt((rel ** 2).mean())), float(np.abs(rel).max())


if __name__ == "__main__":
    C = fit()
    print("coefficients:", [float.hex(c) for c in C])
    print(f"approximation error {approx_err_ulp(C):.3f} ulp (2^-24 relative)")
    m, rms, mx = f32_eval_stats(C)
    print(f"f32 Horner over x in [-12, 0]: mean {m:+.4f}  rms {rms:.4f}  max {mx:.3f} (2^-24 relative)")
