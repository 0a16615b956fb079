"""GPU parity for beam-search decode and alignment utilities (bit-exact vs the C oracle and
the reference's own known answers), through the device C-ABI (torch mirror) and the seven
host-pointer reference symbols."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import decode_cases as dc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _t(x, dt=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    return (t if dt is None else t.to(dt)).to(DEV)


def _eq(gpu_out, ref, keys, ctx=""):
    for k, g in zip(keys, gpu_out):
        g = g.cpu().numpy() if isinstance(g, torch.Tensor) else g
        assert np.array_equal(g, ref[k]), f"{ctx} {k}: gpu={g} ref={ref[k]}"


@pytest.fixture(params=[pytest.param(0, id="rank"), pytest.param(1, marks=pytest.mark.ab, id="select")])
def select_mode(request, gpu):
    """The fused decodes' two step orderings (full rank: the product; selection: forced through
    the A/B build, include/ssnt_tts_c_ab.h) must give identical outputs."""
    if request.param == 0:
        yield 0
        return
    with gpu.use_ab() as ab:
        assert ab.ssnt_fused_decode_select(1) == 0
        yield 1


@pytest.fixture(params=[pytest.param(0, marks=pytest.mark.ab, id="sync"),
                        pytest.param(1, marks=pytest.mark.ab, id="writevalue"),
                        pytest.param(2, id="flagkernel")])
def host_sync(request, gpu):
    """The per-step host symbols' three ways of waiting for their kernel (hipStreamSynchronize,
    a hipStreamWriteValue32 completion word, a completion word written by a flag kernel) must
    return identical outputs."""
    if request.param == 2:  # the product's own mode
        yield 2
        return
    with gpu.use_ab() as ab:
        assert ab.ssnt_set_host_sync(request.param) >= 0
        yield request.param


V1_KEYS = ("prediction", "log_prob", "next_t", "next_u", "next_is_finished", "beam_branch")
V2_KEYS = ("prediction", "log_prob", "next_t", "next_u", "next_is_finished",
           "next_total_duration", "beam_branch")


@pytest.mark.parametrize("seed", range(150))
def test_v1_step_batched(gpu, oracle, seed):
    c = dc.v1_case(seed)
    W = c["h"].shape[1]
    o = oracle.v1_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"])
    g = gpu.beam_search_decode(_t(c["h"]), _t(c["hist"]), _t(c["fin"]), _t(c["t"]), _t(c["u"]),
                               _t(c["input_length"]), W)
    _eq(g, o, V1_KEYS, f"seed={seed}")


@pytest.mark.parametrize("seed", range(150))
def test_tone_step(gpu, oracle, seed):
    c = dc.tone_case(seed)
    B, W, C = c["h"].shape
    o = oracle.tone_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"],
                         c["empty_tone_id"])
    g = gpu.tone_latent_beam_search_decode(_t(c["h"]), _t(c["hist"]), _t(c["fin"]), _t(c["t"]),
                                           _t(c["u"]), _t(c["input_length"]), W, C,
                                           c["empty_tone_id"])
    _eq(g, o, V1_KEYS, f"seed={seed}")


@pytest.mark.parametrize("seed", range(200))
def test_v2_step(gpu, oracle, seed):
    c = dc.v2_case(seed)
    B, W, D = c["h"].shape
    o, rc = oracle.v2_step(c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
                           c["input_length"], c["output_length"], c["zero_duration_id"],
                           c["allow_skip"], c["test_mode"])
    # the reference wrapper zeroes output_length in test mode; pass what the oracle saw
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
    _eq(g, o, V2_KEYS, f"seed={seed}")


@pytest.mark.parametrize("seed", range(40))
def test_reference_host_symbols_v1(gpu, oracle, seed, host_sync):
    # the exact ABI the TF op binds: ssnt_tts_beam_search_decode, batch fixed to 1
    from ssnt_tts_amd import capi
    c = dc.v1_case(seed, B=1)
    W = c["h"].shape[1]
    o = oracle.v1_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"])
    g = capi.ssnt_tts_beam_search_decode(c["h"][0], c["hist"][0], c["fin"][0], c["t"][0],
                                         c["u"][0], int(c["input_length"][0]), W)
    _eq(g, {k: v[0] for k, v in o.items()}, V1_KEYS, f"seed={seed}")


@pytest.mark.parametrize("seed", range(40))
def test_reference_host_symbols_v2_tone(gpu, oracle, seed, host_sync):
    from ssnt_tts_amd import capi
    c = dc.v2_case(seed)
    B, W, D = c["h"].shape
    o, rc = oracle.v2_step(c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
                           c["input_length"], c["output_length"], c["zero_duration_id"],
                           c["allow_skip"], c["test_mode"])
    if rc == 0:
        g = capi.ssnt_tts_v2_beam_search_decode(
            c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
            c["input_length"], c["output_length"], B, W, D, c["zero_duration_id"],
            c["allow_skip"], c["test_mode"])
        _eq(g, o, V2_KEYS, f"v2 seed={seed}")
    c = dc.tone_case(seed)
    B, W, C = c["h"].shape
    o = oracle.tone_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"],
                         c["empty_tone_id"])
    g = capi.tone_latent_beam_search_decode(c["h"], c["hist"], c["fin"], c["t"], c["u"],
                                            c["input_length"], B, W, C, c["empty_tone_id"])
    _eq(g, o, V1_KEYS, f"tone seed={seed}")


def test_host_symbols_zero_copy_stress(gpu, oracle):
    # the product's per-step symbols hand outputs back through coherent zero-copy
    # staging and return when a flag kernel's completion word is seen. Check every output right
    # after each return, over many back-to-back calls of varying shapes (the staging buffer is
    # reused with every size) -- a stale line would show as a wrong beam here.
    from ssnt_tts_amd import capi
    n = 0
    for seed in range(300):
        if seed % 2 == 0:
            c = dc.v1_case(seed, B=1)
            W = c["h"].shape[1]
            o = oracle.v1_step(c["h"], c["hist"], c["fin"], c["t"], c["u"], c["input_length"])
            g = capi.ssnt_tts_beam_search_decode(c["h"][0], c["hist"][0], c["fin"][0], c["t"][0],
                                                 c["u"][0], int(c["input_length"][0]), W)
            _eq(g, {k: v[0] for k, v in o.items()}, V1_KEYS, f"v1 seed={seed}")
        else:
            c = dc.v2_case(seed)
            B, W, D = c["h"].shape
            o, rc = oracle.v2_step(c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"],
                                   c["u"], c["input_length"], c["output_length"],
                                   c["zero_duration_id"], c["allow_skip"], c["test_mode"])
            if rc != 0:
                continue
            g = capi.ssnt_tts_v2_beam_search_decode(
                c["h"], c["hist"], c["fin"], c["total"], c["table"], c["t"], c["u"],
                c["input_length"], c["output_length"], B, W, D, c["zero_duration_id"],
                c["allow_skip"], c["test_mode"])
            _eq(g, o, V2_KEYS, f"v2 seed={seed}")
        n += 1
    assert n > 200


def test_v1_two_step_appendix_b(gpu, golden):
    from ssnt_tts_amd import capi
    fx = golden["v1_two_step"]
    W = fx["beam_width"]
    h = np.array(fx["h_bits"], np.uint32).view(np.float32).reshape(W, 2)
    hist = np.zeros(W, np.float32)
    z = np.zeros(W, np.int32)
    for exp in fx["expected"]:
        p, lp, nt, nu, fin, bb = capi.ssnt_tts_beam_search_decode(h, hist, np.zeros(W, bool), z, z,
                                                                  fx["input_length"], W)
        assert p.tolist() == exp["prediction"]
        assert lp.view(np.uint32).tolist() == exp["log_prob_bits"]
        assert nt.tolist() == exp["next_t"] and nu.tolist() == exp["next_u"]
        assert fin.tolist() == exp["is_finished"] and bb.tolist() == exp["beam_branch"]
        hist = lp


def test_extract_best_beam_branch_known_answer(gpu, golden):
    from ssnt_tts_amd import capi
    fx = golden["extract_best_beam_branch"]
    bb = np.array(fx["beam_branch"], np.int32)
    ob, ot = capi.ssnt_extract_best_beam_branch(fx["best_final_branch"], bb, bb,
                                                fx["beam_width"], fx["max_u"])
    assert ob.tolist() == fx["expected_best_beam_branch"]
    assert ot.tolist() == fx["derived_best_t_history"]
    ob2, ot2 = gpu.extract_best_beam_branch(fx["best_final_branch"], _t(bb), _t(bb), fx["beam_width"])
    assert ob2.cpu().tolist() == fx["expected_best_beam_branch"]
    assert ot2.cpu().tolist() == fx["derived_best_t_history"]


@pytest.mark.parametrize("shape", [(3, 7, 4), (5, 200, 4), (2, 3000, 10), (4, 50, 64)])
def test_order_beam_branch(gpu, oracle, shape):
    from ssnt_tts_amd import capi
    B, T, W = shape
    rng = np.random.default_rng(T)
    bb = rng.integers(0, W, size=(B, T, W)).astype(np.int32)
    fb = rng.integers(0, W, size=(B, W)).astype(np.int32)
    want = oracle.order_beam_branch(fb, bb)
    assert np.array_equal(gpu.order_beam_branch(_t(fb), _t(bb), W).cpu().numpy(), want)
    assert np.array_equal(capi.ssnt_order_beam_branch(fb, bb, B, W, T), want)


def test_upsample_known_answer_and_random(gpu, oracle, golden, host_sync):
    from ssnt_tts_amd import capi
    fx = golden["upsample_source_indexes"]
    d = np.array(fx["duration"], np.int32)
    ol = np.array(fx["output_length"], np.int32)
    out = gpu.upsample_source_indexes(_t(d), _t(ol), -1, fx["beam_width"])
    assert out.cpu().tolist() == fx["expected"]
    assert capi.ssnt_upsample_source_indexes(d, ol, 3, 2, 6, 11).tolist() == fx["expected"]
    rng = np.random.default_rng(0)
    d = rng.integers(0, 6, size=(7, 4, 400)).astype(np.int32)
    d[0, 0, :] = 0
    ol = d.sum(-1).astype(np.int32)
    want, rc = oracle.upsample_source_indexes(d, ol, int(ol.max()))
    assert rc == 0
    assert np.array_equal(gpu.upsample_source_indexes(_t(d), _t(ol), -1, 4).cpu().numpy(), want)
    with pytest.raises(gpu.SsntError):
        gpu.upsample_source_indexes(_t(d), _t(ol + 1), -1, 4)


def test_edit_distance(gpu, oracle, golden):
    from ssnt_tts_amd import capi
    fx = golden["edit_distance_batched"]
    a, b = np.array(fx["a"], np.int32), np.array(fx["b"], np.int32)
    got = gpu.levenshtein_edit_distance(_t(a), _t(b), _t(np.array(fx["a_length"])),
                                        _t(np.array(fx["b_length"])))
    assert got.cpu().tolist() == fx["expected"]
    assert capi.tone_latent_levenshtein_edit_distance(a, b, fx["a_length"], fx["b_length"], 10,
                                                      6).tolist() == fx["expected"]
    for a_, b_, want in golden["edit_distance_pairs"]["cases"]:
        L = max(len(a_), len(b_), 1)
        A = np.full((1, L), -7, np.int32)
        Bv = np.full((1, L), -9, np.int32)
        A[0, :len(a_)] = a_
        Bv[0, :len(b_)] = b_
        assert gpu.levenshtein_edit_distance(_t(A), _t(Bv), _t(np.array([len(a_)])),
                                             _t(np.array([len(b_)]))).item() == want
    rng = np.random.default_rng(1)
    B, L = 64, 150
    a = rng.integers(0, 5, size=(B, L)).astype(np.int32)
    b = rng.integers(0, 5, size=(B, L)).astype(np.int32)
    al = rng.integers(0, L + 1, size=B).astype(np.int32)
    bl = rng.integers(0, L + 1, size=B).astype(np.int32)
    want = oracle.levenshtein(a, b, al, bl)
    assert np.array_equal(gpu.levenshtein_edit_distance(_t(a), _t(b), _t(al), _t(bl)).cpu().numpy(), want)


@pytest.mark.parametrize("tie_rich", [False, True])
def test_lattice_decode_config3(gpu, oracle, tie_rich, select_mode):
    # BASELINE configs[2]: B=256, T=200 decode steps, beam 4, alignment indices bit-exact
    B, T, U, W = 256, 200, 80, 4
    lat = (oracle.synth_tie_rich_log_trans(B, T, U, seed=3) if tie_rich
           else oracle.synth_log_trans(B, T, U, seed=3))
    il = np.full(B, U, np.int32)
    il[::7] = np.random.default_rng(0).integers(1, U, size=len(il[::7]))  # ragged inputs
    want = oracle.v1_lattice_decode(lat, il, W)
    got = gpu.lattice_beam_search_decode(_t(lat), _t(il), W)
    for k, v in want.items():
        assert np.array_equal(got[k].cpu().numpy(), v), k


def test_reference_symbol_aborts_like_a_panic(gpu):
    # v2 with no admissible duration: Rust panics inside an extern fn -> the process aborts
    code = r"""
import sys, numpy as np
sys.path.insert(0, %r)
from ssnt_tts_amd import capi
capi.ssnt_tts_v2_beam_search_decode(np.zeros((1,1,2),np.float32), np.zeros((1,1),np.float32),
    np.zeros((1,1),bool), np.array([[1000]],np.int32), np.array([0,1],np.int32),
    np.zeros((1,1),np.int32), np.zeros((1,1),np.int32), np.array([5],np.int32),
    np.array([20],np.int32), 1, 1, 2, 0, False, False)
print("unreachable")
""" % os.path.join(os.path.dirname(__file__), "..", "ssnt-tts-rust_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "unreachable" not in r.stdout
    assert "could not find a duration sequence" in r.stderr


@pytest.mark.parametrize("shape", [
    (6, 37, 20, 1),    # W = 1, T not a multiple of the 4-row prefetch ring
    (7, 33, 24, 2),    # n = 4 and n = 6: 8-lane candidate replicas with idle lanes in each
    (5, 41, 50, 3),
    (4, 30, 40, 6),    # n = 12 (4 replicas of 16 lanes) and n = 24 (2 replicas of 32)
    (3, 28, 60, 12),
    (5, 70, 130, 4),   # U > 128: rows read from HBM directly (the whole history fits LDS)
    (4, 40, 30, 32),   # 2W = 64 candidates: every lane holds one
    (3, 25, 16, 40),   # W > 32: the LDS step_wave kernel
])
@pytest.mark.parametrize("tie_rich", [False, True])
def test_lattice_decode_paths(gpu, oracle, shape, tie_rich, select_mode):
    # every fused-decode path (register step staged / direct, LDS step) bit-exact vs the oracle
    B, T, U, W = shape
    lat = (oracle.synth_tie_rich_log_trans(B, T, U, seed=T) if tie_rich
           else oracle.synth_log_trans(B, T, U, seed=T))
    il = np.random.default_rng(U).integers(1, U + 1, size=B).astype(np.int32)
    il[0] = U
    want = oracle.v1_lattice_decode(lat, il, W)
    got = gpu.lattice_beam_search_decode(_t(lat), _t(il), W)
    for k, v in want.items():
        assert np.array_equal(got[k].cpu().numpy(), v), k


def test_v1_seven_step_reference_sequence(gpu, oracle, golden, host_sync):
    # ssnt-tts-tensorflow/tests/test_beam_search_op.py:11-34: the reference's only multi-step v1
    # op sequence (W=3, max_t=4), fed step by step through the exact symbol the TF op binds
    # (ssnt_tts_beam_search_decode, host pointers, batch 1) and through the batched device entry;
    # every step's six outputs bit-exact against the oracle, the state carried like the op loop.
    from ssnt_tts_amd import capi
    fx = golden["v1_seven_step_inputs"]
    W, T = fx["beam_width"], fx["max_t"]
    assert len(fx["acts_bits"]) == 7
    hist = np.zeros(W, np.float32)
    t = np.zeros(W, np.int32)
    u = np.zeros(W, np.int32)
    fin = np.zeros(W, bool)
    for step, bits in enumerate(fx["acts_bits"]):
        h = np.array(bits, np.uint32).view(np.float32).reshape(W, 2)
        o = oracle.v1_step(h[None], hist[None], fin[None], t[None], u[None], [T])
        want = {k: v[0] for k, v in o.items()}
        g = capi.ssnt_tts_beam_search_decode(h, hist, fin, t, u, T, W)
        _eq(g, want, V1_KEYS, f"host symbol step={step}")
        gd = gpu.beam_search_decode(_t(h[None]), _t(hist[None]), _t(fin[None]), _t(t[None]),
                                    _t(u[None]), _t(np.array([T], np.int32)), W)
        _eq([x[0] for x in gd], want, V1_KEYS, f"device step={step}")
        hist, t, u, fin = want["log_prob"], want["next_t"], want["next_u"], want["next_is_finished"]
