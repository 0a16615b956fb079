"""Cross-check the C oracle's decode steps against the independent Python restatement
(tests/ref_model.py) on seeded random, tie-rich and edge-case inputs."""
import numpy as np
import pytest

import decode_cases as dc
import ref_model as rm


@pytest.mark.parametrize("seed", range(200))
def test_v1_oracle_vs_python(oracle, seed):
    c = dc.v1_case(seed)
    B, W, _ = c["h"].shape
    o = oracle.v1_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"])
    for b in range(B):
        p = rm.v1_step(c["h"][b], c["hist"][b], c["fin"][b], c["t"][b], c["u"][b],
                       c["input_length"][b], W)
        for k, v in p.items():
            assert np.array_equal(o[k][b], v), (seed, b, k)


@pytest.mark.parametrize("seed", range(200))
def test_tone_oracle_vs_python(oracle, seed):
    c = dc.tone_case(seed)
    B, W, _ = c["h"].shape
    o = oracle.tone_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"],
                         c["empty_tone_id"])
    for b in range(B):
        p = rm.tone_step(c["h"][b], c["hist"][b], c["fin"][b], c["t"][b], c["u"][b],
                         c["input_length"][b], c["empty_tone_id"], W)
        for k, v in p.items():
            assert np.array_equal(o[k][b], v), (seed, b, k)


@pytest.mark.parametrize("seed", range(300))
def test_v2_oracle_vs_python(oracle, seed):
    c = dc.v2_case(seed)
    B, W, _ = c["h"].shape
    o, rc = oracle.v2_step(c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
                           c["input_length"], c["output_length"], c["zero_duration_id"],
                           c["allow_skip"], c["test_mode"])
    any_empty = False
    for b in range(B):
        p = rm.v2_step(c["h"][b], c["hist"][b], c["fin"][b], c["total"][b], c["table"],
                       c["t"][b], c["u"][b], c["input_length"][b], c["output_length"][b],
                       c["zero_duration_id"], c["allow_skip"], c["test_mode"], W)
        if p is None:
            any_empty = True
            continue
        for k, v in p.items():
            assert np.array_equal(o[k][b], v), (seed, b, k)
    assert (rc == 3) == any_empty


def test_v2_diagonal_injection_example(oracle):
    # I=4, O=12, W=2, D=4 at t=1: the diagonal candidate replaces the last slot (src/v2.rs:298-303)
    h = np.log(np.array([[[0.1, 0.2, 0.3, 0.4], [0.4, 0.3, 0.2, 0.1]]], np.float32))
    args = dict(hist=np.zeros((1, 2), np.float32), fin=np.zeros((1, 2), bool),
                total=np.array([[3, 3]], np.int32), table=np.arange(4, dtype=np.int32),
                t=np.array([[1, 1]], np.int32), u=np.array([[1, 1]], np.int32),
                input_length=[4], output_length=[12], zero_duration_id=0, allow_skip=False,
                test_mode=False)
    o, rc = oracle.v2_step(h, **args)
    p = rm.v2_step(h[0], args["hist"][0], args["fin"][0], args["total"][0], args["table"],
                   args["t"][0], args["u"][0], 4, 12, 0, False, False, 2)
    assert rc == 0
    for k, v in p.items():
        assert np.array_equal(o[k][0], v), k
    # the last slot is on the diagonal: tot - O/I * next_t in [-20, 0]
    d = o["next_total_duration"][0, -1] - 12 / 4 * o["next_t"][0, -1]
    assert -20 <= d <= 0


def test_v2_no_candidate_reports_error(oracle):
    # every class outside the band -> assert_ne!(n_results, 0) panics in the reference
    h = np.zeros((1, 1, 2), np.float32)
    o, rc = oracle.v2_step(h, np.zeros((1, 1), np.float32), np.zeros((1, 1), bool),
                           np.array([[1000]], np.int32), np.array([0, 1], np.int32),
                           np.array([[0]], np.int32), np.array([[0]], np.int32), [5], [20], 0,
                           False, False)
    assert rc == 3
