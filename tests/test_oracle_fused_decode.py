"""The oracle's fused multi-step decodes (v2 and tone, configs[4]) against a plain loop of the
per-step oracle (src/v2.rs:221-339, src/tone_latent.rs:144-234) fed back as the next state,
plus order_beam_branch (src/v2_util.rs:6-36): the fused restatement adds no semantics of its
own. CPU only."""
import numpy as np
import pytest

import decode_cases as dc


def _loop(step, B, T, W, v2):
    st = dict(hist=np.zeros((B, W), np.float32), fin=np.zeros((B, W), bool),
              t=np.zeros((B, W), np.int32), u=np.zeros((B, W), np.int32),
              total=np.zeros((B, W), np.int32))
    hist = {}
    for s in range(T):
        o = step(s, st)
        if o is None:
            return None
        for k, v in o.items():
            hist.setdefault(k, []).append(v)
        st = dict(hist=o["log_prob"], fin=o["next_is_finished"], t=o["next_t"], u=o["next_u"],
                  total=o["next_total_duration"] if v2 else st["total"])
    return {k: np.stack(v, axis=1) for k, v in hist.items()}


def _paths(oracle, o, W, v2):
    B, T, _ = o["beam_branch"].shape
    fb = np.tile(np.arange(W, dtype=np.int32), (B, 1))
    ordered = oracle.order_beam_branch(fb, o["beam_branch"])
    bi = np.arange(B)[:, None, None]
    si = np.arange(T)[None, None, :]
    pp = o["prediction"][bi, si, ordered]
    res = dict(ordered_beam_branch=ordered, path_prediction=pp)
    if v2:
        tot = o["next_total_duration"][bi, si, ordered]
        prev = np.concatenate([np.zeros((B, W, 1), np.int32), tot[:, :, :-1]], axis=2)
        res["duration"] = tot - prev
    return res


@pytest.mark.parametrize("seed", range(120))
def test_fused_v2_equals_step_loop(oracle, seed):
    c = dc.fused_v2_case(seed)
    B, T, W, D = c["logits"].shape
    ol = np.zeros(B, np.int32) if c["test_mode"] else c["output_length"]

    def step(s, st):
        o, rc = oracle.v2_step(c["logits"][:, s], st["hist"], st["fin"], st["total"], c["table"],
                               st["t"], st["u"], c["input_length"], ol, c["zero_duration_id"],
                               c["allow_skip"], c["test_mode"])
        return None if rc != 0 else o

    ref = _loop(step, B, T, W, True)
    got, rc = oracle.v2_lattice_decode(c["logits"], c["table"], c["input_length"],
                                       c["output_length"], c["zero_duration_id"], c["allow_skip"],
                                       c["test_mode"])
    if ref is None:
        assert rc == 3
        return
    assert rc == 0
    ref.update(_paths(oracle, ref, W, True))
    for k, v in ref.items():
        assert np.array_equal(got[k], v), (seed, k)


@pytest.mark.parametrize("seed", range(120))
def test_fused_tone_equals_step_loop(oracle, seed):
    c = dc.fused_tone_case(seed)
    B, T, W, C = c["logits"].shape

    def step(s, st):
        return oracle.tone_step(c["logits"][:, s], st["hist"], st["fin"], st["t"], st["u"],
                                c["input_length"], c["empty_tone_id"])

    ref = _loop(step, B, T, W, False)
    ref.update(_paths(oracle, ref, W, False))
    got = oracle.tone_lattice_decode(c["logits"], c["input_length"], c["empty_tone_id"])
    for k, v in ref.items():
        assert np.array_equal(got[k], v), (seed, k)


@pytest.mark.parametrize("seed", range(3))
def test_config5_v2_synthetic_path_is_found(oracle, seed):
    """configs[4] sizes: the sampled duration path (sum == O, inside the band) is the best
    beam, every final slot lands exactly on O, and the durations upsample cleanly."""
    B, I, O, D, W = 16, 400, 2000, 16, 4
    d = oracle.synth_durations(B, I, O, D, seed=seed)
    assert (d.sum(1) == O).all() and d.min() >= 1 and d.max() <= D - 1
    lg = oracle.synth_v2_logits(d, W, D, seed=seed + 10)
    o, rc = oracle.v2_lattice_decode(lg, np.arange(D), np.full(B, I), np.full(B, O), 0, False,
                                     False)
    assert rc == 0
    assert np.array_equal(o["path_prediction"][:, 0], d)
    assert (o["next_total_duration"][:, -1] == O).all()
    assert (o["duration"].sum(-1) == O).all()
    up, urc = oracle.upsample_source_indexes(o["duration"], o["next_total_duration"][:, -1], O)
    assert urc == 0 and (up >= 0).all()
