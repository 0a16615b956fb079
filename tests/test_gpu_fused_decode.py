"""GPU parity of the fused multi-step decodes (BASELINE configs[4]: v2 + tone_latent at
I=400 input positions, O=2000 frames, D=16, C=5, W=4, B=64) against the oracle's fused
restatement, which tests/test_oracle_fused_decode.py pins to a loop of the per-step oracle.
Bit-exact on every per-step output and every path output; "no candidate" (the reference's
panic, src/v2.rs:292) must be reported for the same inputs."""
import numpy as np
import pytest
import torch

import decode_cases as dc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

V2_OUT = ("prediction", "log_prob", "next_t", "next_u", "next_is_finished", "next_total_duration",
          "beam_branch", "ordered_beam_branch", "path_prediction", "duration")
TONE_OUT = ("prediction", "log_prob", "next_t", "next_u", "next_is_finished", "beam_branch",
            "ordered_beam_branch", "path_prediction")


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


@pytest.fixture(autouse=True, params=[pytest.param(0, id="rank"), pytest.param(1, marks=pytest.mark.ab, id="select")])
def select_mode(request, gpu):
    """The fused decodes' two step orderings (full rank: the product; selection: forced through
    the A/B build, include/ssnt_tts_c_ab.h) must give identical outputs."""
    if request.param == 0:
        yield 0
        return
    with gpu.use_ab() as ab:
        assert ab.ssnt_fused_decode_select(1) == 0
        yield 1


def _same(g, o, keys, ctx):
    for k in keys:
        gv = g[k].cpu().numpy()
        if not np.array_equal(gv, o[k]):
            bad = np.argwhere(gv != o[k])
            raise AssertionError(f"{ctx} {k}: {len(bad)} mismatches, first at {bad[0].tolist()}")


def _v2(gpu, oracle, lg, table, il, ol, zid, skip, test_mode, ctx, upsample=False):
    o, rc = oracle.v2_lattice_decode(lg, table, il, ol, zid, skip, test_mode)
    args = (_t(lg), _t(table), _t(il), _t(ol), lg.shape[2], zid, skip, test_mode)
    if rc == 3:
        with pytest.raises(gpu.SsntError):
            gpu.v2_lattice_beam_search_decode(*args)
        return None
    assert rc == 0
    g = gpu.v2_lattice_beam_search_decode(*args, upsample=upsample)
    _same(g, o, V2_OUT, ctx)
    return g, o


def _config5(oracle, seed, B=64, I=400, O=2000, D=16, W=4, ragged=False, **kw):
    rng = np.random.default_rng(seed)
    if ragged:
        Ib = rng.integers(I // 2, I + 1, size=B).astype(np.int32)
        Ob = (Ib * (O // I) + rng.integers(-20, 21, size=B)).astype(np.int32)
    else:
        Ib, Ob = np.full(B, I, np.int32), np.full(B, O, np.int32)
    d = oracle.synth_durations(B, Ib, Ob, D, seed=seed)
    d = np.pad(d, ((0, 0), (0, I - d.shape[1])))
    return oracle.synth_v2_logits(d, W, D, seed=seed + 100, **kw), Ib, Ob, d


@pytest.mark.parametrize("seed", range(3))
def test_v2_config5_full_size(gpu, oracle, seed):
    """B=64 T=I=400 O=2000 D=16 W=4 (W*D = 64: one candidate per lane), logits peaked on a
    sampled duration path that sums to O: the band and exact-length rules decide every step."""
    D = 16
    lg, il, ol, d = _config5(oracle, seed)
    g, o = _v2(gpu, oracle, lg, np.arange(D, dtype=np.int32), il, ol, 0, False, False,
               f"seed={seed}", upsample=True)
    assert np.array_equal(o["path_prediction"][:, 0], d)  # the sampled path is the best beam
    assert (o["next_total_duration"][:, -1] == 2000).all()
    up, urc = oracle.upsample_source_indexes(o["duration"], o["next_total_duration"][:, -1], 2000)
    assert urc == 0
    assert np.array_equal(g["upsampled_source_indexes"].cpu().numpy(), up)


def test_v2_config5_test_mode(gpu, oracle):
    lg, il, ol, _ = _config5(oracle, 7)
    _v2(gpu, oracle, lg, np.arange(16, dtype=np.int32), il, ol, 0, False, True, "test_mode")


def test_v2_config5_tie_rich(gpu, oracle):
    lg, il, ol, _ = _config5(oracle, 8, tie_rich=True)
    _v2(gpu, oracle, lg, np.arange(16, dtype=np.int32), il, ol, 0, False, False, "tie-rich")


def test_v2_config5_ragged_lengths(gpu, oracle):
    """Per-utterance I in [200, 400] and O near 5 I: finished beams keep padding until T=400."""
    lg, il, ol, _ = _config5(oracle, 9, ragged=True)
    _v2(gpu, oracle, lg, np.arange(16, dtype=np.int32), il, ol, 0, False, False, "ragged")


def test_v2_config5_allow_skip(gpu, oracle):
    lg, il, ol, _ = _config5(oracle, 10, margin=6.0)
    _v2(gpu, oracle, lg, np.arange(16, dtype=np.int32), il, ol, 0, True, False, "allow_skip")


def test_v2_no_candidate_is_reported(gpu, oracle):
    """A weak peak loses the exact-length path in some utterances: both sides report it."""
    lg, il, ol, _ = _config5(oracle, 2, margin=2.0)
    o, rc = oracle.v2_lattice_decode(lg, np.arange(16), il, ol, 0, False, False)
    assert rc == 3
    _v2(gpu, oracle, lg, np.arange(16, dtype=np.int32), il, ol, 0, False, False, "no-candidate")


@pytest.mark.parametrize("W,D", [(5, 16), (8, 16), (3, 30)])
def test_v2_more_candidates_than_lanes(gpu, oracle, W, D):
    """W*D > 64: the any-size LDS kernel, at I=400 O=2000."""
    lg, il, ol, _ = _config5(oracle, 11 + W, B=8, D=D, W=W)
    _v2(gpu, oracle, lg, np.arange(D, dtype=np.int32), il, ol, 0, False, False, f"W={W} D={D}")


@pytest.mark.parametrize("seed", range(150))
def test_v2_fused_random(gpu, oracle, seed):
    c = dc.fused_v2_case(seed)
    _v2(gpu, oracle, c["logits"], c["table"], c["input_length"], c["output_length"],
        c["zero_duration_id"], c["allow_skip"], c["test_mode"], f"seed={seed}")


PRODUCT_TONE_WAVES = 1  # fused_decode.hip kToneWaves


@pytest.fixture(params=[pytest.param(w, id=f"tone{w}w", marks=() if w == PRODUCT_TONE_WAVES else pytest.mark.ab)
                        for w in (1, 2, 4)])
def tone_waves(request, gpu):
    """Tone's 20-candidate rank split over 1, 2 or 4 waves (the product's choice, and the others
    forced through the A/B build): identical outputs."""
    if request.param == PRODUCT_TONE_WAVES:
        yield request.param
        return
    with gpu.use_ab() as ab:
        assert ab.ssnt_fused_decode_tone_waves(request.param) == 0
        yield request.param


def _tone(gpu, oracle, lg, il, eid, ctx):
    o = oracle.tone_lattice_decode(lg, il, eid)
    g = gpu.tone_latent_lattice_beam_search_decode(_t(lg), _t(il), lg.shape[2], eid)
    _same(g, o, TONE_OUT, ctx)


@pytest.mark.parametrize("tie_rich", [False, True])
def test_tone_config5(gpu, oracle, tone_waves, tie_rich):
    """B=64 T=I=400 C=5 W=4 (20 candidates), ragged input lengths up to the step count."""
    B, T, W, C = 64, 400, 4, 5
    lg = oracle.synth_tone_logits(B, T, W, C, seed=20 + tie_rich, tie_rich=tie_rich)
    il = np.random.default_rng(21).integers(T // 2, T + 1, size=B).astype(np.int32)
    il[:8] = T
    _tone(gpu, oracle, lg, il, 0, f"tie_rich={tie_rich}")


def test_tone_more_candidates_than_lanes(gpu, oracle):
    B, T, W, C = 4, 400, 16, 5
    lg = oracle.synth_tone_logits(B, T, W, C, seed=22, tie_rich=True)
    _tone(gpu, oracle, lg, np.full(B, 390, np.int32), 0, "W*C=80")


@pytest.mark.parametrize("seed", range(150))
def test_tone_fused_random(gpu, oracle, tone_waves, seed):
    c = dc.fused_tone_case(seed)
    _tone(gpu, oracle, c["logits"], c["input_length"], c["empty_tone_id"], f"seed={seed}")


V2_STEP = ("prediction", "log_prob", "next_t", "next_u", "next_is_finished",
           "next_total_duration", "beam_branch")


@pytest.mark.parametrize("W,D", [(4, 16), (5, 16), (2, 32), (8, 16)])
@pytest.mark.parametrize("seed", range(10))
def test_v2_single_step_long(gpu, oracle, W, D, seed):
    """One v2 step at I=400, O=2000 with W*D = 64 and > 64 candidates."""
    c = dc.v2_case_long(seed, W, D)
    ol = np.zeros_like(c["output_length"]) if c["test_mode"] else c["output_length"]
    o, rc = oracle.v2_step(c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
                           c["input_length"], ol, c["zero_duration_id"], c["allow_skip"],
                           c["test_mode"])
    args = (_t(c["h"]), _t(c["hist"]), _t(c["fin"]), _t(c["total"]), _t(c["table"]), _t(c["t"]),
            _t(c["u"]), _t(c["input_length"]), _t(c["output_length"]), W, D,
            c["zero_duration_id"], c["allow_skip"], c["test_mode"])
    if rc == 3:
        with pytest.raises(gpu.SsntError):
            gpu.ssnt_tts_v2_beam_search_decode(*args)
        return
    g = gpu.ssnt_tts_v2_beam_search_decode(*args)
    for k, v in zip(V2_STEP, g):
        assert np.array_equal(v.cpu().numpy(), o[k]), (seed, k)


@pytest.mark.parametrize("kind", ["step_v1", "step_v2", "fused_v1", "fused_v2", "fused_tone"])
def test_nan_inputs_stay_in_range(gpu, oracle, kind):
    """NaN log-probs are outside the parity contract, but the rank must stay a
    permutation: every output index in range, and the same total order (NaN below -inf) as the
    oracle, so the outputs still match it."""
    rng = np.random.default_rng(0)
    if kind == "step_v1":
        c = dc.v1_case(3, B=4, W=6, max_t=5)
        c["h"][:, ::2, 0] = np.nan
        c["hist"][:, 1] = np.nan
        o = oracle.v1_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"])
        g = gpu.beam_search_decode(_t(c["h"]), _t(c["hist"]), _t(c["fin"]), _t(c["t"]), _t(c["u"]),
                                   _t(c["input_length"]), 6)
        bb = g[5].cpu().numpy()
        assert ((bb >= 0) & (bb < 6)).all()
        assert np.array_equal(bb, o["beam_branch"])
        return
    if kind == "step_v2":
        c = dc.v2_case_long(1, 4, 16)
        c["h"][:, :, 3:7] = np.nan
        ol = np.zeros_like(c["output_length"]) if c["test_mode"] else c["output_length"]
        o, rc = oracle.v2_step(c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
                               c["input_length"], ol, c["zero_duration_id"], c["allow_skip"],
                               c["test_mode"])
        g = gpu.ssnt_tts_v2_beam_search_decode(
            _t(c["h"]), _t(c["hist"]), _t(c["fin"]), _t(c["total"]), _t(c["table"]), _t(c["t"]),
            _t(c["u"]), _t(c["input_length"]), _t(c["output_length"]), 4, 16,
            c["zero_duration_id"], c["allow_skip"], c["test_mode"], check=False)
        bb = g[6].cpu().numpy()
        assert ((bb >= 0) & (bb < 4)).all()
        if rc == 0:
            assert np.array_equal(bb, o["beam_branch"])
        return
    if kind == "fused_v1":
        lat = oracle.synth_log_trans(8, 40, 16, seed=1)
        lat[:, 5:9, 3:6, :] = np.nan
        il = np.full(8, 16, np.int32)
        o = oracle.v1_lattice_decode(lat, il, 4)
        g = gpu.lattice_beam_search_decode(_t(lat), _t(il), 4)
        for k in ("beam_branch", "best_beam_branch"):
            v = g[k].cpu().numpy()
            assert ((v >= 0) & (v < 4)).all()
            assert np.array_equal(v, o[k]), k
        return
    if kind == "fused_v2":
        lg, il, ol, _ = _config5(oracle, 3, B=8)
        lg[:, 50:60, :, ::3] = np.nan
        o, rc = oracle.v2_lattice_decode(lg, np.arange(16), il, ol, 0, False, True)
        g = gpu.v2_lattice_beam_search_decode(_t(lg), _t(np.arange(16, dtype=np.int32)), _t(il),
                                              _t(ol), 4, 0, False, True)
        assert rc == 0
        _same(g, o, ("beam_branch", "ordered_beam_branch", "prediction"), "nan v2")
        return
    lg = oracle.synth_tone_logits(8, 50, 4, 5, seed=4)
    lg[:, 10:20, 1] = np.nan
    il = np.full(8, 50, np.int32)
    o = oracle.tone_lattice_decode(lg, il, 0)
    g = gpu.tone_latent_lattice_beam_search_decode(_t(lg), _t(il), 4, 0)
    _same(g, o, ("beam_branch", "ordered_beam_branch", "prediction"), "nan tone")


# Long decodes: the register kernel's two other history layouts. WHOLE (every per-step record in
# LDS as 16-byte records, one flush after the loop) holds while 16*T*W fits beside the rank
# buffers (T*W <= ~9300 for one wave, ~9000 for the four-wave v2 step; RegLayout in
# fused_decode.hip); past that the records are flushed every 32 steps with the (parent, aux[,
# total]) history kept in LDS for the in-launch backtrace; past ~150 KB of history (nh*4*T*W
# bytes) the history stays in the global outputs and k_fused_paths backtraces from there.
@pytest.mark.parametrize("T,U,W,ctx", [
    (3000, 80, 4, "chunked flush, history in LDS, staged rows"),
    (2600, 300, 4, "chunked flush, history in LDS, rows from HBM"),
    (700, 40, 32, "history beyond LDS: k_fused_paths"),
])
@pytest.mark.parametrize("tie_rich", [False, True])
def test_v1_long_history_layouts(gpu, oracle, T, U, W, ctx, tie_rich):
    B = 5
    lat = (oracle.synth_tie_rich_log_trans(B, T, U, seed=T + W) if tie_rich
           else oracle.synth_log_trans(B, T, U, seed=T + W))
    il = np.random.default_rng(T).integers(U // 2, U + 1, size=B).astype(np.int32)
    il[0] = U
    want = oracle.v1_lattice_decode(lat, il, W)
    got = gpu.lattice_beam_search_decode(_t(lat), _t(il), W)
    for k, v in want.items():
        g = got[k].cpu().numpy()
        if not np.array_equal(g, v):
            bad = np.argwhere(g != v)
            raise AssertionError(f"{ctx} {k}: {len(bad)} mismatches, first at {bad[0].tolist()}")


def test_v2_long_chunked_flush(gpu, oracle):
    # I=2800 steps at W=4, D=16 (T*W = 11200): chunked flush with the 3-array history in LDS;
    # the band and exact-length rules decide every step (O = 5 I)
    lg, il, ol, _ = _config5(oracle, 31, B=4, I=2800, O=14000, D=16, W=4)
    _v2(gpu, oracle, lg, np.arange(16, dtype=np.int32), il, ol, 0, False, False, "v2 I=2800")


def test_v2_history_beyond_lds(gpu, oracle):
    # W=16, D=4 (64 candidates, one per lane), I=1000 test-mode steps: 3*4*T*W = 192 KB of
    # history > LDS, so the paths come from k_fused_paths over the global outputs
    B, I, W, D = 3, 1000, 16, 4
    lg = oracle.synth_tone_logits(B, I, W, D, seed=32)
    il = np.array([1000, 990, 700], np.int32)
    _v2(gpu, oracle, lg, np.arange(D, dtype=np.int32), il, np.zeros(B, np.int32), 0, True, True,
        "v2 W=16 D=4 I=1000 test_mode")


@pytest.mark.parametrize("T,W,C,ctx", [
    (3000, 4, 5, "chunked flush, history in LDS"),
    (500, 64, 1, "history beyond LDS: k_fused_paths"),
])
def test_tone_long_history_layouts(gpu, oracle, tone_waves, T, W, C, ctx):
    B = 4
    lg = oracle.synth_tone_logits(B, T, W, C, seed=T + C, tie_rich=True)
    il = np.random.default_rng(T).integers(T // 2, T + 1, size=B).astype(np.int32)
    il[0] = T
    _tone(gpu, oracle, lg, il, 0, ctx)
