"""Independent references for the lattice forward-backward -- TEST INFRASTRUCTURE.

* brute_force: enumerate every monotone emit/shift path (tiny lattices only).
* torch_dp: dense float64 log-domain DP in torch; gradients by autograd.
Both restate DESIGN.md "Lattice semantics"  independently of the C oracle.
"""
import itertools
import math

import numpy as np


def brute_force(lt, S, P, lo=None, terminal=True):
    """lt (T,U,2) f64-able; returns (loss, grad (T,U,2), grad_obs (T,U))."""
    T, U, _ = lt.shape
    lt = lt.astype(np.float64)
    lo = None if lo is None else lo.astype(np.float64)
    scores, uses = [], []
    if S >= 1 and P >= 1 and S >= P:
        for ks in itertools.product((0, 1), repeat=S - 1):
            p = 0
            sc = 0.0 if lo is None else lo[0, 0]
            used = []
            ok = True
            for s, k in enumerate(ks):
                if p + k > P - 1:
                    ok = False
                    break
                sc += lt[s, p, k]
                used.append((s, p, k))
                p += k
                if lo is not None:
                    sc += lo[s + 1, p]
            if not ok or p != P - 1:
                continue
            if terminal:
                sc += lt[S - 1, P - 1, 0]
                used.append((S - 1, P - 1, 0))
            scores.append(sc)
            uses.append(used)
    g = np.zeros((T, U, 2))
    go = np.zeros((T, U))
    if not scores:
        return math.inf, g, go
    m = max(scores)
    logZ = m + math.log(sum(math.exp(x - m) for x in scores))
    for sc, used in zip(scores, uses):
        w = math.exp(sc - logZ)
        cells = [(0, 0)]
        for (s, p, k) in used:
            g[s, p, k] -= w
            if s + 1 < S:
                cells.append((s + 1, p + k))
        for c in cells:
            go[c] -= w
    return -logZ, g, go


def torch_dp(lt, S, P, lo=None, terminal=True):
    """Dense log-domain DP in float64 torch; returns (loss, grad, grad_obs) via autograd."""
    import torch
    T, U, _ = lt.shape
    x = torch.tensor(lt, dtype=torch.float64, requires_grad=True)
    o = None if lo is None else torch.tensor(lo, dtype=torch.float64, requires_grad=True)
    NEG = -1e30  # finite stand-in for log(0): torch.logaddexp(-inf, -inf) has a NaN gradient
    ninf = torch.tensor(NEG, dtype=torch.float64)
    if not (S >= 1 and P >= 1 and S >= P):
        return math.inf, np.zeros((T, U, 2)), np.zeros((T, U))
    a = torch.full((P,), NEG, dtype=torch.float64)
    a = torch.cat([(o[0, 0] if o is not None else torch.zeros((), dtype=torch.float64)).reshape(1), a[1:]])
    for s in range(1, S):
        stay = a + x[s - 1, :P, 0]
        shift = torch.cat([ninf.reshape(1), a[:-1] + x[s - 1, :P - 1, 1]])
        a = torch.logaddexp(stay, shift)
        if o is not None:
            a = a + o[s, :P]
    logZ = a[P - 1] + (x[S - 1, P - 1, 0] if terminal else 0.0)
    loss = -logZ
    loss.backward()
    g = x.grad.numpy().copy()
    go = np.zeros((T, U)) if o is None else o.grad.numpy().copy()
    return float(loss.detach()), g, go
