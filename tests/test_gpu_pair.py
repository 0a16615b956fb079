"""GPU parity for the pair kernel (csrc/fwd_bwd_pair.hip): variant 12, U <= 128 without log_obs. Bit-exact against the oracle's pair recurrence (oracle.fwd_bwd_xf(pair=True),
ORACLE_PAIR in oracle/ssnt_oracle.c), which tests/test_oracle_fwd_bwd.py pins to the float64
DP and to brute-force path enumeration within the north_star tolerance.

Covers both step-length parities (S-1 odd: the backward chain starts with one ordinary step),
the smallest lattices (S = 1..5: cut at 0, one pair, the terminal pair alone), ragged batches,
both flags, -inf transitions, the debug rows, K = 1 and 2 lane widths, both ring depths
(8 pair slots for U <= 80, 4 above), the narrow form (U odd, 4/8-byte aligned tensors) and the
workspace form (rows beyond LDS)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F_TERM, F_ZINF = 1, 2


@pytest.fixture(autouse=True)
def pair_variant(gpu):
    """The pair kernel is selected with the A/B build's ssnt_fwd_bwd_set_variant(12) (the product keeps
    the one-step streaming kernel, which measured faster: DESIGN.md 5.1a)."""
    with gpu.use_ab() as ab:
        assert ab.ssnt_fwd_bwd_set_variant(12) == 0
        yield


def _run(gpu, lt, S, P, flags=F_TERM, debug=True, shift=0):
    dev = torch.device("cuda:0")
    x = torch.from_numpy(lt).to(dev)
    out = None
    if shift:
        B, T, U, _ = lt.shape
        flat = torch.zeros(lt.size + shift, dtype=torch.float32, device=dev)
        flat[shift:] = x.ravel()
        x = flat[shift:].view(B, T, U, 2)
        gflat = torch.full((lt.size + shift,), 7.0, dtype=torch.float32, device=dev)
        out = {"grad": gflat[shift:].view(B, T, U, 2)}
    r = gpu.ssnt_fwd_bwd(x, torch.tensor(S, dtype=torch.int32, device=dev),
                         torch.tensor(P, dtype=torch.int32, device=dev),
                         terminal_emit=bool(flags & F_TERM), zero_infinity=bool(flags & F_ZINF),
                         debug=debug, check=True, out=out)
    kern = gpu.last_fwd_bwd_kernel()
    assert kern.startswith("k_fwd_bwd_pair<"), kern
    return {k: v.cpu().numpy() for k, v in r.items() if k != "status"}, kern


def _assert_bit_exact(g, o, keys):
    for k in keys:
        a, b = g[k], o[k]
        assert a.shape == b.shape, k
        same = (a == b) | (np.isnan(a) & np.isnan(b))
        if not np.all(same):
            idx = np.argwhere(~same)[:5]
            raise AssertionError(f"{k}: {np.sum(~same)} cells differ, e.g. {idx.tolist()} "
                                 f"gpu={a[tuple(idx[0])]} oracle={b[tuple(idx[0])]}")


DBG = ["loss", "grad", "log_alpha", "log_beta"]


@pytest.mark.parametrize("T", [1, 2, 3, 4, 5, 6, 7, 8, 9, 16, 17])
def test_small_lattices_every_parity(gpu, oracle, T):
    # every S in 1..T with P from 1..S: cut at 0 / 2, the terminal pair alone, S-1 odd and even
    U = 6
    cases = [(s, p) for s in range(1, T + 1) for p in range(1, min(s, U) + 1)]
    B = len(cases)
    lt = oracle.synth_log_trans(B, T, U, seed=T)
    S = [c[0] for c in cases]
    P = [c[1] for c in cases]
    for flags in (F_TERM, 0):
        g, _ = _run(gpu, lt, S, P, flags=flags)
        o = oracle.fwd_bwd_xf(lt, S, P, flags=flags, debug=True, pair=True)
        _assert_bit_exact(g, o, DBG)


@pytest.mark.parametrize("shape", [(1, 50, 20), (3, 37, 64), (4, 60, 65), (5, 90, 80), (3, 41, 81),
                                   (2, 64, 127), (2, 70, 128), (6, 200, 80), (4, 199, 80)])
def test_full_lengths(gpu, oracle, shape):
    B, T, U = shape
    lt = oracle.synth_log_trans(B, T, U, seed=B * 1000 + T)
    S, P = [T] * B, [min(U, T)] * B
    g, _ = _run(gpu, lt, S, P)
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True, pair=True)
    _assert_bit_exact(g, o, DBG)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("flags", [F_TERM, 0, F_TERM | F_ZINF])
@pytest.mark.parametrize("U", [33, 80, 100])
def test_ragged_and_edges(gpu, oracle, seed, flags, U):
    rng = np.random.default_rng(seed)
    B, T = 9, 48
    P = rng.integers(1, U + 1, size=B)
    P = np.minimum(P, T)
    S = np.array([rng.integers(max(1, p), T + 1) for p in P])
    S[0], P[0] = 1, 1          # single cell
    S[1], P[1] = 10, 12        # infeasible (S < P)
    S[2], P[2] = 0, 1          # empty
    S[3], P[3] = T, min(U, T)  # full
    S[4], P[4] = 20, 20        # S == P: one path
    lt = oracle.synth_log_trans(B, T, U, seed=seed)
    lt[5, :, 3, 1] = -np.inf   # log(0) transitions
    lt[6, 10:30, :, 0] = -np.inf
    g, _ = _run(gpu, lt, S, P, flags=flags)
    o = oracle.fwd_bwd_xf(lt, S, P, flags=flags, debug=True, pair=True)
    _assert_bit_exact(g, o, DBG)


def test_config2_full_size(gpu, oracle):
    # BASELINE configs[1]: B=256 T=200 U=80 -- the bench workload, bit-exact, posterior mass 1
    B, T, U = 256, 200, 80
    lt = oracle.synth_log_trans(B, T, U, seed=0)
    S, P = [T] * B, [U] * B
    g, kern = _run(gpu, lt, S, P, debug=False)
    assert "LDS=1" in kern and "NV=0" in kern
    o = oracle.fwd_bwd_xf(lt, S, P, pair=True)
    _assert_bit_exact(g, o, ["loss", "grad"])
    occ = -g["grad"][:, :T - 1].sum(axis=(2, 3))
    assert np.max(np.abs(occ - 1.0)) < 1e-4


@pytest.mark.parametrize("shift", [1, 2, 4])
@pytest.mark.parametrize("U", [80, 81, 127, 33])
def test_offsets_narrow_form(gpu, oracle, shift, U):
    B, T = 5, max(90, U + 10)
    lt = oracle.synth_log_trans(B, T, U, seed=shift + U)
    rng = np.random.default_rng(shift)
    P = [U] + [int(x) for x in rng.integers(1, U + 1, size=B - 1)]
    S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
    g, kern = _run(gpu, lt, S, P, shift=shift)
    K = 1 if U <= 64 else 2
    if shift % 4 or U % K:  # the narrow form: U % K != 0 or tensors below 16-byte alignment
        assert "NV=1" in kern, kern
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True, pair=True)
    _assert_bit_exact(g, o, DBG)


@pytest.mark.parametrize("shape", [(3, 320, 80), (2, 300, 128), (2, 900, 40)])
def test_workspace_form(gpu, oracle, shape):
    B, T, U = shape
    rng = np.random.default_rng(T)
    lt = oracle.synth_log_trans(B, T, U, seed=T)
    P = [U] + [int(x) for x in rng.integers(1, U + 1, size=B - 1)]
    S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
    g, kern = _run(gpu, lt, S, P)
    assert "LDS=0" in kern, kern
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True, pair=True)
    _assert_bit_exact(g, o, DBG)


def test_more_workgroups_than_cus_with_loss_sum(gpu, oracle):
    dev = torch.device("cuda:0")
    B, T, U = 2048, 24, 16
    lt = oracle.synth_log_trans(B, T, U, seed=5)
    x = torch.from_numpy(lt).to(dev)
    sl = torch.full((B,), T, dtype=torch.int32, device=dev)
    pl = torch.full((B,), U, dtype=torch.int32, device=dev)
    o = oracle.fwd_bwd_xf(lt, [T] * B, [U] * B, pair=True)
    for _ in range(2):
        r = gpu.ssnt_fwd_bwd(x, sl, pl, loss_sum=True, check=True)
        assert gpu.last_fwd_bwd_kernel().startswith("k_fwd_bwd_pair<")
        assert np.array_equal(r["loss"].cpu().numpy(), o["loss"])
        assert np.array_equal(r["grad"].cpu().numpy(), o["grad"])
