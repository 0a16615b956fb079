"""GPU parity for F4, the v2 duration-class forward-backward (through libssnt_tts_c.so).

Bar: BIT-EXACT against the split-exponent C oracle (oracle/ssnt_oracle.c "F4") on loss,
gradients and the debug rows; the oracle itself is pinned to float64 and to brute-force path
enumeration (tests/test_oracle_v2_fwd_bwd.py). At the configs[4] size (B=64, I=400, O=2000,
D=16) the same bit-exact check runs, plus the posterior-mass property (sum_i posterior = 1)."""
import numpy as np
import pytest
import torch

from f4_cases import random_case

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _run(gpu, logits, table, I, O, zid=0, allow_skip=True, test_mode=False, max_total=None,
         zero_infinity=False, debug=True):
    t = lambda a, dt: torch.as_tensor(np.asarray(a), dtype=dt, device=DEV)  # noqa: E731
    r = gpu.v2_fwd_bwd(t(logits, torch.float32), t(table, torch.int32), t(I, torch.int32),
                       t(O, torch.int32), zid, allow_skip=allow_skip, test_mode=test_mode,
                       max_total=max_total, zero_infinity=zero_infinity, debug=debug, check=True)
    return {k: v.cpu().numpy() for k, v in r.items() if k != "status"}


def _same(g, o, keys):
    for k in keys:
        a, b = g[k], o[k]
        assert a.shape == b.shape, k
        ok = (a == b) | (np.isnan(a) & np.isnan(b))
        if not ok.all():
            idx = np.argwhere(~ok)[:5]
            raise AssertionError(f"{k}: {int((~ok).sum())} cells differ, e.g. {idx.tolist()} "
                                 f"gpu={a[tuple(idx[0])]} oracle={b[tuple(idx[0])]}")


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("mode", ["band", "test_mode", "no_skip"])
def test_small_bit_exact(gpu, oracle, seed, mode):
    rng = np.random.default_rng(seed)
    B, Imax, D = 7, 9, 5
    logits, I, O = random_case(rng, B, Imax, D)
    table = np.arange(D, dtype=np.int32)
    test_mode, allow_skip = mode == "test_mode", mode != "no_skip"
    mt = int(O.max()) + (9 if test_mode else 0)
    g = _run(gpu, logits, table, I, O, 0, allow_skip, test_mode, mt)
    o = oracle.v2_fwd_bwd(logits, table, I, O, mt, 0, allow_skip, test_mode, debug=True)
    _same(g, o, ["loss", "grad", "log_alpha", "log_beta"])


@pytest.mark.parametrize("test_mode", [False, True])
def test_medium_ragged_bit_exact(gpu, oracle, test_mode):
    B, Imax, D = 12, 60, 8
    d = oracle.synth_durations(B, Imax, 4 * Imax, D, seed=3)
    logits = oracle.synth_v2_step_logits(d, D, seed=4)
    rng = np.random.default_rng(5)
    I = rng.integers(Imax // 2, Imax + 1, size=B).astype(np.int32)
    I[0] = Imax
    O = np.array([int(d[b, :I[b]].sum()) for b in range(B)], np.int32)
    table = np.arange(D, dtype=np.int32)
    mt = int(O.max()) + (40 if test_mode else 3)
    g = _run(gpu, logits, table, I, O, 0, True, test_mode, mt)
    o = oracle.v2_fwd_bwd(logits, table, I, O, mt, 0, True, test_mode, debug=True)
    _same(g, o, ["loss", "grad", "log_alpha", "log_beta"])
    assert np.all(np.isfinite(g["loss"]))


def test_edges(gpu, oracle):
    rng = np.random.default_rng(11)
    B, Imax, D = 7, 6, 4
    logits, _, _ = random_case(rng, B, Imax, D)
    table = np.array([0, 1, 2, 3], np.int32)
    I = np.array([6, 0, 4, 6, 3, 6, 5], np.int32)
    O = np.array([19, 5, 9, 16, 6, 14, 12], np.int32)  # > max_total, I=0, ok, no moves, ok, overrun, ok
    logits[3] = -np.inf
    logits[6, 2, :2] = np.nan  # NaN log-probs: dropped moves
    logits[4, 1, 1] = np.inf   # clamped to XF_LOG_MAX
    for zi in (False, True):
        g = _run(gpu, logits, table, I, O, 0, True, False, 18, zero_infinity=zi)
        o = oracle.v2_fwd_bwd(logits, table, I, O, 18, 0, True, False,
                              flags=oracle.FLAG_ZERO_INFINITY if zi else 0, debug=True)
        _same(g, o, ["loss", "grad", "log_alpha", "log_beta"])


def test_no_skip_zero_class_is_never_used(gpu, oracle):
    rng = np.random.default_rng(2)
    logits, I, O = random_case(rng, 4, 8, 4)
    table = np.array([0, 1, 2, 3], np.int32)
    g = _run(gpu, logits, table, I, O, zid=0, allow_skip=False, max_total=int(O.max()))
    fin = np.isfinite(g["loss"])
    assert not g["grad"][fin][:, :, 0].any()


def test_config5_bit_exact(gpu, oracle):
    # BASELINE configs[4] v2 shape: B=64, I=400, O=2000, D=16, duration_table = [0..15]
    B, I, Ot, D = 64, 400, 2000, 16
    d = oracle.synth_durations(B, I, Ot, D, seed=0)
    logits = oracle.synth_v2_step_logits(d, D, seed=1)
    table = np.arange(D, dtype=np.int32)
    il, ol = np.full(B, I, np.int32), np.full(B, Ot, np.int32)
    g = _run(gpu, logits, table, il, ol, 0, False, False, Ot, debug=False)
    assert np.all(np.isfinite(g["loss"]))
    mass = -g["grad"].sum(-1)
    assert np.max(np.abs(mass - 1.0)) < 1e-4
    o = oracle.v2_fwd_bwd(logits, table, il, ol, Ot, 0, False, False)
    _same(g, o, ["loss", "grad"])


def test_autograd(gpu, oracle):
    rng = np.random.default_rng(8)
    logits, I, O = random_case(rng, 3, 7, 4)
    table = np.arange(4, dtype=np.int32)
    x = torch.from_numpy(logits).to(DEV).requires_grad_(True)
    loss = gpu.v2_duration_loss(x, torch.from_numpy(table).to(DEV), torch.from_numpy(I).to(DEV),
                                torch.from_numpy(O).to(DEV), 0, True, False, None, True)
    w = torch.tensor([1.0, 0.5, 2.0], device=DEV)
    (loss * w).sum().backward()
    o = oracle.v2_fwd_bwd(logits, table, I, O, int(O.max()), 0, True, False,
                          flags=oracle.FLAG_ZERO_INFINITY)
    assert np.array_equal(loss.detach().cpu().numpy(), o["loss"])
    assert np.array_equal(x.grad.cpu().numpy(), o["grad"] * np.array([1.0, 0.5, 2.0], np.float32)[:, None, None])


def test_negative_duration_is_reported(gpu):
    logits = np.zeros((2, 3, 3), np.float32)
    with pytest.raises(gpu.SsntError):
        _run(gpu, logits, [0, -1, 2], [3, 3], [4, 4], max_total=6)


@pytest.mark.parametrize("zero_infinity", [False, True])
def test_band_mode_output_length_beyond_max_total(gpu, oracle, zero_infinity):
    # band mode with O > max_total (e.g. I=100, O=1000, max_total=20): the band windows of the
    # early rows are wider than the band-sized row capacity, and the exact final total can never
    # be reached, so the lattice is empty: loss +inf (0 under zero_infinity), grads 0, rows -inf
    rng = np.random.default_rng(21)
    B, Imax, D = 3, 100, 8
    logits = rng.standard_normal((B, Imax, D)).astype(np.float32)
    table = np.arange(D, dtype=np.int32)
    I = np.array([100, 100, 40], np.int32)
    O = np.array([1000, 300, 21], np.int32)
    g = _run(gpu, logits, table, I, O, 0, True, False, 20, zero_infinity=zero_infinity)
    o = oracle.v2_fwd_bwd(logits, table, I, O, 20, 0, True, False,
                          flags=oracle.FLAG_ZERO_INFINITY if zero_infinity else 0, debug=True)
    _same(g, o, ["loss", "grad", "log_alpha", "log_beta"])
    assert np.all(g["loss"] == (0.0 if zero_infinity else np.inf))
    assert not g["grad"].any()


F4_TABLES = [  # (name, duration_table): both cell forms and every class padding of the sweep
    ("long_durations", [0, 3, 70, 5, 100, 2]),  # dmax 100 > 64: the clamped cell form
    ("shuffled16", [7, 0, 12, 3, 9, 1, 15, 4, 2, 11, 6, 14, 8, 13, 10, 5]),
    ("d20", list(range(0, 60, 3))),              # 32 class slots
    ("d40", [(5 * i) % 64 for i in range(40)]),  # 64 class slots, 32-step weight chunks
]


@pytest.mark.parametrize("test_mode", [False, True])
@pytest.mark.parametrize("name,table", F4_TABLES, ids=[t[0] for t in F4_TABLES])
def test_duration_tables_bit_exact(gpu, oracle, name, table, test_mode):
    # Non-identity duration tables, long ones beyond the sweep's padded row buffers, and I past
    # two weight chunks (the staged chunks); utterance 4's band moves further per step than the
    # longest duration (every cell of a row then reads outside the previous window: exact zeros)
    table = np.array(table, np.int32)
    D = len(table)
    B, Imax = 5, 150
    rng = np.random.default_rng(D)
    logits = rng.standard_normal((B, Imax, D)).astype(np.float32) * np.float32(1.5)
    m = logits.max(-1, keepdims=True)
    logits = (logits - (m + np.log(np.exp(logits - m).sum(-1, keepdims=True)))).astype(np.float32)
    I = np.array([150, 149, 97, 70, 20], np.int32)
    O = np.array([int(table[rng.integers(0, D, size=i)].sum()) for i in I], np.int32)
    O[4] = int(I[4]) * (int(table.max()) + 30)
    mt = int(O[:4].max()) + (7 if test_mode else 0)
    if test_mode:
        O[4] = min(int(O[4]), mt)
    g = _run(gpu, logits, table, I, O, 0, True, test_mode, mt)
    o = oracle.v2_fwd_bwd(logits, table, I, O, mt, 0, True, test_mode, debug=True)
    _same(g, o, ["loss", "grad", "log_alpha", "log_beta"])
    assert np.isfinite(g["loss"][:4]).any()
