"""F4 oracle (v2 duration-class fwd-bwd): the split-exponent restatement pinned against an
independent float64 DP and against brute-force enumeration of class sequences. The reference
has no such function: "parity unpinned" by the reference -- its move rules are
the v2 decode's (src/v2.rs:94-166), checked here move by move."""
import numpy as np
import pytest

import oracle as O
from f4_cases import brute_force, random_case

TABLE4 = np.array([0, 1, 2, 3], np.int32)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("mode", ["band", "test_mode", "no_skip"])
def test_brute_force_small(seed, mode):
    rng = np.random.default_rng(seed)
    B, Imax, D = 3, 5, 4
    logits, I, Ol = random_case(rng, B, Imax, D)
    test_mode = mode == "test_mode"
    allow_skip = mode != "no_skip"
    max_total = int(Ol.max()) + (6 if test_mode else 0)
    f64 = O.v2_fwd_bwd_f64(logits, TABLE4, I, Ol, max_total, 0, allow_skip, test_mode)
    xf = O.v2_fwd_bwd(logits, TABLE4, I, Ol, max_total, 0, allow_skip, test_mode)
    for b in range(B):
        loss, grad = brute_force(logits[b], TABLE4, int(I[b]), int(Ol[b]), max_total, 0,
                                 allow_skip, test_mode)
        if np.isinf(loss):
            assert np.isinf(f64["loss"][b]) and np.isinf(xf["loss"][b])
            assert not xf["grad"][b].any()
            continue
        assert abs(f64["loss"][b] - loss) < 1e-9 * max(1.0, abs(loss))
        np.testing.assert_allclose(f64["grad"][b], grad, atol=1e-12)
        assert abs(float(xf["loss"][b]) - loss) < 1e-5 + 2 ** -22 * abs(loss)
        np.testing.assert_allclose(xf["grad"][b], grad, atol=2e-6)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("test_mode", [False, True])
def test_xf_vs_f64_medium(seed, test_mode):
    rng = np.random.default_rng(100 + seed)
    B, Imax, D = 6, 40, 8
    table = np.arange(D, dtype=np.int32)
    d = O.synth_durations(B, Imax, 4 * Imax, D, seed=seed)
    logits = O.synth_v2_step_logits(d, D, seed=seed)
    I = np.full(B, Imax, np.int32)
    I[1] = Imax - 7
    Ol = d.sum(1).astype(np.int32)
    Ol[1] = int(d[1, :I[1]].sum())
    max_total = int(Ol.max()) + (20 if test_mode else 0)
    f64 = O.v2_fwd_bwd_f64(logits, table, I, Ol, max_total, 0, True, test_mode)
    xf = O.v2_fwd_bwd(logits, table, I, Ol, max_total, 0, True, test_mode)
    assert np.all(np.isfinite(xf["loss"]))
    np.testing.assert_allclose(xf["loss"], f64["loss"], rtol=2e-6, atol=1e-5)
    np.testing.assert_allclose(xf["grad"], f64["grad"], atol=1e-5)
    # posterior mass 1 per step
    for b in range(B):
        mass = -xf["grad"][b, :I[b]].sum(-1)
        assert np.max(np.abs(mass - 1.0)) < 1e-4
        assert not xf["grad"][b, I[b]:].any()


def test_infeasible_and_edges():
    rng = np.random.default_rng(3)
    B, Imax, D = 5, 6, 4
    logits, _, _ = random_case(rng, B, Imax, D)
    I = np.array([6, 0, 4, 6, 3], np.int32)
    Ol = np.array([100, 5, 9, 16, 6], np.int32)  # > max_total; I=0; ok; no moves; ok
    logits[3, :, :] = -np.inf  # no moves at all
    out = O.v2_fwd_bwd(logits, TABLE4, I, Ol, 20, 0, True, False)
    assert np.isinf(out["loss"][0]) and np.isinf(out["loss"][1]) and np.isinf(out["loss"][3])
    assert np.isfinite(out["loss"][2]) and np.isfinite(out["loss"][4])
    # a short output the overrun rule forbids (src/v2.rs:106-111): (I-1)*3 > O
    short = O.v2_fwd_bwd(logits[:1], TABLE4, [6], [14], 20, 0, True, False)
    assert np.isinf(short["loss"][0])
    zi = O.v2_fwd_bwd(logits, TABLE4, I, Ol, 20, 0, True, False, flags=O.FLAG_ZERO_INFINITY)
    assert zi["loss"][0] == 0.0 and zi["loss"][3] == 0.0
    assert not out["grad"][[0, 1, 3]].any()
    with pytest.raises(RuntimeError):
        O.v2_fwd_bwd(logits, np.array([0, -1, 2, 3], np.int32), I, Ol, 20, 0, True, False)


def test_nan_logits_are_dropped_moves():
    rng = np.random.default_rng(9)
    logits, I, Ol = random_case(rng, 2, 5, 4)
    lg = logits.copy()
    lg[:, 2, 1] = np.nan
    ref = logits.copy()
    ref[:, 2, 1] = -np.inf
    a = O.v2_fwd_bwd(lg, TABLE4, I, Ol, int(Ol.max()), 0, True, False, debug=True)
    b = O.v2_fwd_bwd(ref, TABLE4, I, Ol, int(Ol.max()), 0, True, False, debug=True)
    for k in a:
        assert np.array_equal(a[k], b[k])
