"""Seeded decode-step input generators shared by the oracle cross-checks and the GPU parity
tests (tie-rich values, finished beams, out-of-range t, duplicated beams)."""
import numpy as np

PROBS = np.array([0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9], np.float32)


def _logits(rng, shape, tie_rich):
    if tie_rich:
        return np.log(rng.choice(PROBS, size=shape).astype(np.float32)).astype(np.float32)
    return (rng.standard_normal(shape).astype(np.float32) * np.float32(2.0)).astype(np.float32)


def v1_case(seed, B=None, W=None, max_t=None):
    rng = np.random.default_rng(seed)
    B = B or int(rng.integers(1, 6))
    W = W or int(rng.integers(1, 9))
    max_t = max_t if max_t is not None else int(rng.integers(1, 8))
    tie = bool(rng.integers(0, 2))
    h = _logits(rng, (B, W, 2), tie)
    # histories drawn from a small set so equal log-probs (dedup) happen often
    base = _logits(rng, (B, max(1, W // 2)), True)
    hist = base[:, rng.integers(0, base.shape[1], size=W)].astype(np.float32)
    if rng.random() < 0.3:
        hist[:] = 0.0
    t = rng.integers(-1, max_t + 2, size=(B, W)).astype(np.int32)
    u = rng.integers(0, 20, size=(B, W)).astype(np.int32)
    if rng.random() < 0.5:  # duplicated beams (all beams equal, as at decode start)
        t[:] = t[:, :1]
        u[:] = u[:, :1]
        h[:] = h[:, :1]
    fin = rng.random((B, W)) < 0.2
    il = np.full(B, max_t, np.int32)
    return dict(h=h, hist=hist, fin=fin, t=t, u=u, input_length=il)


def tone_case(seed):
    rng = np.random.default_rng(seed + 1000)
    B, W, C = int(rng.integers(1, 5)), int(rng.integers(1, 7)), int(rng.integers(1, 7))
    tie = bool(rng.integers(0, 2))
    h = _logits(rng, (B, W, C), tie)
    hist = _logits(rng, (B, W), True)
    if rng.random() < 0.4:
        hist[:] = 0.0
        h[:] = h[:, :1]
    il = rng.integers(0, 6, size=B).astype(np.int32)
    t = rng.integers(-1, 8, size=(B, W)).astype(np.int32)
    u = rng.integers(0, 9, size=(B, W)).astype(np.int32)
    fin = rng.random((B, W)) < 0.2
    return dict(h=h, hist=hist, fin=fin, t=t, u=u, input_length=il,
                empty_tone_id=int(rng.integers(0, C)))


def v2_case(seed):
    """A v2 state in which candidates usually exist: O >= 3(I-1), totals near the diagonal."""
    rng = np.random.default_rng(seed + 2000)
    B, W, D = int(rng.integers(1, 5)), int(rng.integers(1, 6)), int(rng.integers(2, 9))
    I = rng.integers(2, 12, size=B).astype(np.int32)
    O = (3 * (I - 1) + rng.integers(0, 30, size=B)).astype(np.int32)
    table = np.arange(D, dtype=np.int32)
    tie = bool(rng.integers(0, 2))
    h = _logits(rng, (B, W, D), tie)
    hist = _logits(rng, (B, W), True)
    t = np.zeros((B, W), np.int32)
    tot = np.zeros((B, W), np.int32)
    for b in range(B):
        t[b] = rng.integers(0, I[b], size=W)
        diag = O[b] / I[b] * t[b]
        tot[b] = np.maximum(0, (diag + rng.integers(-6, 4, size=W))).astype(np.int32)
    if rng.random() < 0.3:
        t[:, -1] = I[:, None][:, 0] - 1  # last position -> exact-length rule
    u = rng.integers(0, 40, size=(B, W)).astype(np.int32)
    fin = rng.random((B, W)) < 0.15
    return dict(h=h, hist=hist, fin=fin, total=tot, table=table, t=t, u=u, input_length=I,
                output_length=O, zero_duration_id=int(rng.integers(0, D)),
                allow_skip=bool(rng.integers(0, 2)), test_mode=bool(rng.random() < 0.25))


def v2_case_long(seed, W, D, B=3, I=400, O=2000):
    """A single v2 step at the configs[4] lengths (I=400, O=2000): beams at random positions
    with totals near the diagonal, so band / exact-length / diagonal rules all fire."""
    rng = np.random.default_rng(seed + 3000)
    table = np.arange(D, dtype=np.int32)
    tie = bool(rng.integers(0, 2))
    h = _logits(rng, (B, W, D), tie)
    hist = _logits(rng, (B, W), True)
    t = rng.integers(0, I, size=(B, W)).astype(np.int32)
    if rng.random() < 0.5:
        t[:, : max(1, W // 2)] = I - 1
    diag = O / I * t
    tot = np.maximum(0, diag + rng.integers(-8, 6, size=(B, W))).astype(np.int32)
    tot[t == I - 1] = O - rng.integers(0, D, size=int((t == I - 1).sum()))
    u = t.copy()
    fin = rng.random((B, W)) < 0.1
    return dict(h=h, hist=hist, fin=fin, total=tot, table=table, t=t, u=u,
                input_length=np.full(B, I, np.int32), output_length=np.full(B, O, np.int32),
                zero_duration_id=0, allow_skip=bool(rng.integers(0, 2)),
                test_mode=bool(rng.random() < 0.25))


def fused_v2_case(seed):
    """Small fused v2 decode: per-step logits (B,T,W,D), ragged I <= T, O >= 3(I-1)."""
    rng = np.random.default_rng(seed + 4000)
    B, W, D = int(rng.integers(1, 5)), int(rng.integers(1, 6)), int(rng.integers(2, 10))
    if rng.random() < 0.3:  # more candidates than lanes: the any-size kernel
        W, D = int(rng.integers(5, 9)), int(rng.integers(14, 20))
    T = int(rng.integers(1, 24))
    I = rng.integers(1, T + 1, size=B).astype(np.int32)
    O = (3 * np.maximum(I - 1, 0) + rng.integers(0, 3 * D, size=B)).astype(np.int32)
    tie = bool(rng.integers(0, 2))
    logits = _logits(rng, (B, T, W, D), tie)
    table = np.arange(D, dtype=np.int32)
    if rng.random() < 0.3:
        table = rng.integers(0, D + 3, size=D).astype(np.int32)
    return dict(logits=logits, table=table, input_length=I, output_length=O,
                zero_duration_id=int(rng.integers(-1, D + 1)), allow_skip=bool(rng.integers(0, 2)),
                test_mode=bool(rng.random() < 0.3))


def fused_tone_case(seed):
    rng = np.random.default_rng(seed + 5000)
    B, W, C = int(rng.integers(1, 5)), int(rng.integers(1, 8)), int(rng.integers(1, 8))
    if rng.random() < 0.25:
        W, C = int(rng.integers(10, 17)), int(rng.integers(5, 9))
    T = int(rng.integers(1, 24))
    I = rng.integers(0, T + 2, size=B).astype(np.int32)
    tie = bool(rng.integers(0, 2))
    return dict(logits=_logits(rng, (B, T, W, C), tie), input_length=I,
                empty_tone_id=int(rng.integers(-1, C + 1)))
