"""Pin the C oracle to every known answer the reference's own tests hold."""
import numpy as np


def _f32(bits):
    return np.array(bits, dtype=np.uint32).view(np.float32)


def test_extract_best_beam_branch_known_answer(oracle, golden):
    # tests/test_decoding.rs:120-130 (asserted), t_history = beam_branch
    fx = golden["extract_best_beam_branch"]
    bb = np.array(fx["beam_branch"], np.int32)
    out, out_t = oracle.extract_best_beam_branch(fx["best_final_branch"], bb, bb)
    assert out.tolist() == fx["expected_best_beam_branch"]
    assert out_t.tolist() == fx["derived_best_t_history"]


def test_v1_two_step_appendix_b(oracle, golden):
    # tests/test_decoding.rs:13-51: two rounds from (t=0,u=0), W=3, T=4
    fx = golden["v1_two_step"]
    W = fx["beam_width"]
    h = _f32(fx["h_bits"]).reshape(1, W, 2)
    hist = np.zeros((1, W), np.float32)
    zeros = np.zeros((1, W), np.int32)
    fin = np.zeros((1, W), bool)
    for exp in fx["expected"]:
        o = oracle.v1_step(h, hist, fin, zeros, zeros, [fx["input_length"]])
        assert o["prediction"][0].tolist() == exp["prediction"]
        assert o["log_prob"][0].view(np.uint32).tolist() == exp["log_prob_bits"]
        assert o["next_t"][0].tolist() == exp["next_t"]
        assert o["next_u"][0].tolist() == exp["next_u"]
        assert o["next_is_finished"][0].tolist() == exp["is_finished"]
        assert o["beam_branch"][0].tolist() == exp["beam_branch"]
        hist = o["log_prob"]  # round 2: t, u reset to 0 as the Rust test does


def test_upsample_known_answer(oracle, golden):
    # ssnt-tts-tensorflow/tests/test_upsample_source_indexes.py:40-53 (asserted)
    fx = golden["upsample_source_indexes"]
    d = np.array(fx["duration"], np.int32)
    ol = np.array(fx["output_length"], np.int32)
    out, rc = oracle.upsample_source_indexes(d, ol, int(ol.max()), fill=fx["out_of_range_source_index"])
    assert rc == 0
    assert out.tolist() == fx["expected"]


def test_upsample_duration_mismatch_is_an_error(oracle):
    d = np.array([[[1, 2]]], np.int32)
    out, rc = oracle.upsample_source_indexes(d, np.array([[4]], np.int32), 4)
    assert rc == 4  # src/v2_util.rs:58 assert_eq! -> panic


def test_edit_distance_pairs(oracle, golden):
    # tests/test_edit_distance.rs:9-63 (asserted, Kaldi cases)
    for a, b, want in golden["edit_distance_pairs"]["cases"]:
        L = max(len(a), len(b), 1)
        A = np.full((1, L), -7, np.int32)
        Bv = np.full((1, L), -9, np.int32)
        A[0, :len(a)] = a
        Bv[0, :len(b)] = b
        assert oracle.levenshtein(A, Bv, [len(a)], [len(b)])[0] == want


def test_edit_distance_batched(oracle, golden):
    # tests/test_edit_distance.rs:65-106 (asserted, padded batch)
    fx = golden["edit_distance_batched"]
    got = oracle.levenshtein(np.array(fx["a"]), np.array(fx["b"]), fx["a_length"], fx["b_length"])
    assert got.tolist() == fx["expected"]


def test_v1_seven_step_sequence_matches_python_restatement(oracle, golden):
    # ssnt-tts-tensorflow/tests/test_beam_search_op.py:11-50 (no assertions in the reference):
    # the C oracle and the independent Python restatement must agree on every step.
    from ref_model import v1_step as py_v1
    fx = golden["v1_seven_step_inputs"]
    W, T = fx["beam_width"], fx["max_t"]
    hist = np.zeros(W, np.float32)
    t = np.zeros(W, np.int32)
    u = np.zeros(W, np.int32)
    fin = np.zeros(W, bool)
    for bits in fx["acts_bits"]:
        h = _f32(bits).reshape(W, 2)
        o = oracle.v1_step(h[None], hist[None], fin[None], t[None], u[None], [T])
        p = py_v1(h, hist, fin, t, u, T, W)
        for k in ("prediction", "log_prob", "next_t", "next_u", "next_is_finished", "beam_branch"):
            assert np.array_equal(o[k][0], p[k]), k
        hist, t, u, fin = o["log_prob"][0], o["next_t"][0], o["next_u"][0], o["next_is_finished"][0]
