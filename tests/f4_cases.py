"""Shared F4 (v2 duration-class fwd-bwd) cases and the brute-force path enumerator."""
import itertools

import numpy as np


def band(t, I, O):
    """total_duration_bounds (src/v2.rs:94-104), f32 arithmetic restated with numpy."""
    f = np.float32
    diag = f(O) / f(I) * f(t + 1)
    lb = int(max(f(diag - f(O) * f(0.05)), f(0.0)))
    ub = int(min(f(diag + f(O) * f(0.1)), f(O)))
    return lb, ub


def move_ok(t, new_total, i, I, O, X, zid, allow_skip, test_mode):
    """decode_beam_at's keep rule for one candidate (src/v2.rs:127-164)."""
    if not allow_skip and i == zid:
        return False
    if new_total < 0 or new_total >= X:
        return False
    if test_mode:
        return True
    lb, ub = band(t, I, O)
    if new_total < lb or new_total > ub:
        return False
    if (I - (t + 1)) * 3 > O:
        return False
    return t != I - 1 or new_total == O


def brute_force(logits, table, I, O, max_total, zid, allow_skip, test_mode):
    """Every class sequence of one utterance: (loss, grad) in float64 (-inf-safe)."""
    Imax, D = logits.shape
    X = max_total + 1
    Z = 0.0
    post = np.zeros((Imax, D))
    for seq in itertools.product(range(D), repeat=I):
        tot, ok, lp = 0, True, 0.0
        for t, i in enumerate(seq):
            tot += int(table[i])
            if not move_ok(t, tot, i, I, O, X, zid, allow_skip, test_mode) or not logits[t, i] >= -1e6:
                ok = False
                break
            lp += float(logits[t, i])
        if not ok:
            continue
        p = np.exp(lp)
        Z += p
        for t, i in enumerate(seq):
            post[t, i] += p
    if Z == 0.0:
        return np.inf, np.zeros((Imax, D))
    return -np.log(Z), -post / Z


def random_case(rng, B, Imax, D, max_dur=None):
    """Random per-utterance lengths whose exact-total paths exist (durations near O/I)."""
    max_dur = D - 1 if max_dur is None else max_dur
    I = rng.integers(1, Imax + 1, size=B).astype(np.int32)
    O = np.array([int(rng.integers(i, i * max_dur + 1)) for i in I], np.int32)
    logits = rng.standard_normal((B, Imax, D)).astype(np.float32) * np.float32(1.5)
    m = logits.max(-1, keepdims=True)
    logits = (logits - (m + np.log(np.exp(logits - m).sum(-1, keepdims=True)))).astype(np.float32)
    return logits, I, O
