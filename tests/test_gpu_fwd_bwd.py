"""GPU parity for the lattice forward-backward (through libssnt_tts_c.so).

Bar: BIT-EXACT against the split-exponent C oracle (oracle/ssnt_oracle.c) on loss, gradients,
obs gradients and log-alpha / log-beta -- which itself is pinned to float64 truth within the
north_star tolerance (tests/test_oracle_fwd_bwd.py: 1e-5 abs on gradients, 1e-5 + 2^-23|x| on
log values). At full BASELINE sizes the same bit-exact check runs (the multi-threaded oracle
finishes in seconds), plus size-independent properties (posterior mass 1 per step).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F_TERM, F_ZINF = 1, 2


@pytest.fixture(autouse=True, params=[0, 1, 2], ids=["default", "simple", "segmented"])
def kernel_variant(request, gpu):
    """Every parity case runs on every product kernel (they must be bit-identical): the product
    library's own dispatch, and the two-wave / segmented kernels -- which the product dispatches
    for other shapes and alignments -- forced through the A/B build (include/ssnt_tts_c_ab.h)."""
    if request.param == 0:
        yield 0
        return
    with gpu.use_ab() as ab:
        assert ab.ssnt_fwd_bwd_set_variant(request.param) == 0
        yield request.param
        ab.ssnt_fwd_bwd_set_variant(0)


def _run_gpu(gpu, lt, S, P, lo=None, flags=F_TERM, debug=True):
    dev = torch.device("cuda:0")
    r = gpu.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.tensor(S, dtype=torch.int32, device=dev),
                         torch.tensor(P, dtype=torch.int32, device=dev),
                         None if lo is None else torch.from_numpy(lo).to(dev),
                         terminal_emit=bool(flags & F_TERM), zero_infinity=bool(flags & F_ZINF),
                         debug=debug, check=True)
    return {k: v.cpu().numpy() for k, v in r.items() if k != "status"}


def _assert_bit_exact(g, o, keys):
    for k in keys:
        a, b = g[k], o[k]
        assert a.shape == b.shape, k
        same = (a == b) | (np.isnan(a) & np.isnan(b))
        if not np.all(same):
            idx = np.argwhere(~same)[:5]
            raise AssertionError(f"{k}: {np.sum(~same)} cells differ, e.g. {idx.tolist()} "
                                 f"gpu={a[tuple(idx[0])]} oracle={b[tuple(idx[0])]}")


SHAPES = [  # (B, T, U) -- covers K = 1, 2, 4, 8 lanes-per-position layouts and odd U
    (1, 50, 20),    # BASELINE configs[0]
    (3, 37, 64),    # K=1 upper edge
    (4, 60, 65),    # K=2, odd U
    (5, 90, 80),    # K=2, the config-2 position count
    (3, 45, 130),   # K=4
    (2, 30, 300),   # K=8
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("obs", [False, True])
def test_bit_exact_full_lengths(gpu, oracle, shape, obs):
    B, T, U = shape
    lt = oracle.synth_log_trans(B, T, U, seed=B * 1000 + T)
    lo = (np.random.default_rng(T).standard_normal((B, T, U)) * 15 - 40).astype(np.float32) if obs else None
    S, P = [T] * B, [U] * B
    if T < U:
        P = [T] * B
    g = _run_gpu(gpu, lt, S, P, lo)
    o = oracle.fwd_bwd_xf(lt, S, P, log_obs=lo, debug=True)
    keys = ["loss", "grad", "log_alpha", "log_beta"] + (["grad_obs"] if obs else [])
    _assert_bit_exact(g, o, keys)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("flags", [F_TERM, 0, F_TERM | F_ZINF])
def test_bit_exact_ragged_and_edges(gpu, oracle, seed, flags):
    rng = np.random.default_rng(seed)
    B, T, U = 9, 48, 33
    P = rng.integers(1, U + 1, size=B)
    S = np.array([rng.integers(max(1, p), T + 1) for p in P])
    S[0], P[0] = 1, 1          # single cell
    S[1], P[1] = 10, 12        # infeasible (S < P)
    S[2], P[2] = 0, 1          # empty
    S[3], P[3] = T, U          # full
    S[4], P[4] = 20, 20        # S == P: one path
    lt = oracle.synth_log_trans(B, T, U, seed=seed)
    lt[5, :, 3, 1] = -np.inf   # log(0) transitions
    lt[6, 10:30, :, 0] = -np.inf
    g = _run_gpu(gpu, lt, S, P, flags=flags)
    o = oracle.fwd_bwd_xf(lt, S, P, flags=flags, debug=True)
    _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


def test_streaming_kernel_is_the_default_at_config2(gpu, kernel_variant):
    # the product's dispatch runs the streaming kernel at BASELINE configs[1] (and configs[0])
    if kernel_variant != 0:
        pytest.skip("the product's own dispatch")
    dev = torch.device("cuda:0")
    for (B, T, U) in [(2, 200, 80), (1, 50, 20)]:
        x = torch.zeros((B, T, U, 2), device=dev)
        gpu.ssnt_fwd_bwd(x, torch.full((B,), T, dtype=torch.int32, device=dev),
                         torch.full((B,), U, dtype=torch.int32, device=dev), check=True)
        assert gpu.last_fwd_bwd_kernel().startswith("k_fwd_bwd_stream<"), gpu.last_fwd_bwd_kernel()


def test_workspace_mode_long_rows(gpu, oracle):
    # T*U*8 bytes > LDS budget -> rows live in the global workspace
    B, T, U = 3, 320, 80
    lt = oracle.synth_log_trans(B, T, U, seed=9)
    S, P = [320, 250, 200], [80, 70, 33]
    g = _run_gpu(gpu, lt, S, P)
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True)
    _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


def test_config2_full_size_bit_exact(gpu, oracle):
    # BASELINE configs[1]: B=256 T=200 U=80, f32 loss + grad
    B, T, U = 256, 200, 80
    lt = oracle.synth_log_trans(B, T, U, seed=0)
    S, P = [T] * B, [U] * B
    g = _run_gpu(gpu, lt, S, P, debug=False)
    o = oracle.fwd_bwd_xf(lt, S, P)
    _assert_bit_exact(g, o, ["loss", "grad"])
    occ = -g["grad"][:, :T - 1].sum(axis=(2, 3))  # posterior mass per transition step
    assert np.max(np.abs(occ - 1.0)) < 1e-4


def _run_debug64(gpu, lt, S, P, flags=F_TERM):
    dev = torch.device("cuda:0")
    r = gpu.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.tensor(S, dtype=torch.int32, device=dev),
                         torch.tensor(P, dtype=torch.int32, device=dev),
                         terminal_emit=bool(flags & F_TERM), zero_infinity=bool(flags & F_ZINF),
                         debug64=True, check=True)
    return {k: v.cpu().numpy() for k, v in r.items() if k != "status"}


def _check_debug64(g, lt, S, P, oracle, flags=F_TERM, f64=True):
    """GPU float64 outputs vs (1) the float64 logs of the oracle's own split-exponent state (the
    same bits: only the two float64 log() implementations differ) and (2) the float64 DP within
    the north_star 1e-5 abs."""
    st = oracle.fwd_bwd_xf_state(lt, S, P, flags=flags)
    assert np.array_equal(g["grad"], st["grad"]), "gradients of the debug64 launch"
    for k, gk in (("alpha", "log_alpha"), ("beta", "log_beta")):
        want = oracle.xf_log64(st[k])
        fin = np.isfinite(want)
        assert np.array_equal(np.isfinite(g[gk]), fin), k
        assert np.all(np.isneginf(g[gk][~fin])), k
        assert np.max(np.abs(g[gk][fin] - want[fin]), initial=0.0) <= 1e-9, k
    zw = -oracle.xf_log64(st["z"])
    fz = st["z"]["m"] != 0
    assert np.max(np.abs(g["loss"][fz] - zw[fz]), initial=0.0) <= 1e-9
    assert np.array_equal(g["loss"][~fz], st["loss"][~fz].astype(np.float64))  # +inf / 0 as f32
    if not f64:
        return None
    ref = oracle.fwd_bwd_f64(lt, S, P, flags=flags)
    worst = {}
    for gk in ("log_alpha", "log_beta"):
        y = ref[gk]
        fin = np.isfinite(y)
        assert np.array_equal(np.isfinite(g[gk]), fin), gk
        worst[gk] = float(np.max(np.abs(g[gk][fin] - y[fin]), initial=0.0))
    fl = np.isfinite(ref["loss"])
    worst["loss"] = float(np.max(np.abs(g["loss"][fl] - ref["loss"][fl]), initial=0.0))
    # the north_star tolerance on log-alpha / log-beta (and the loss, a log value too)
    assert max(worst.values()) <= 1e-5, worst
    return worst


@pytest.mark.parametrize("config", ["configs1_full_batch", "configs4_two_utterances"])
def test_debug64_north_star_tolerance(gpu, oracle, kernel_variant, config):
    # log-alpha / log-beta / loss formed in float64 on the GPU from the
    # kernel's split-exponent state (ssnt_fwd_bwd_debug64_device) are within 1e-5 abs of the
    # float64 DP at BASELINE configs[1]'s full batch and two full configs[4] utterances
    B, T, U, seed = {"configs1_full_batch": (256, 200, 80, 0),
                     "configs4_two_utterances": (2, 2000, 400, 4)}[config]
    lt = oracle.synth_log_trans(B, T, U, seed=seed)
    S, P = [T] * B, [U] * B
    g = _run_debug64(gpu, lt, S, P)
    worst = _check_debug64(g, lt, S, P, oracle)
    print(config, gpu.last_fwd_bwd_kernel(), worst)


def test_debug64_all_config5_utterances(gpu, oracle, kernel_variant):
    # every one of the 64 configs[4] utterances (B=64 T=2000 U=400, the seed of the long-form
    # parity test) through the product dispatch: float64 log-alpha / log-beta / loss within the
    # north_star 1e-5 abs of the float64 DP (CPU study: 8.7e-6 at worst)
    if kernel_variant != 0:
        pytest.skip("the product's own dispatch")
    B, T, U = 64, 2000, 400
    lt = oracle.synth_log_trans(B, T, U, seed=4)
    S, P = [T] * B, [U] * B
    g = _run_debug64(gpu, lt, S, P)
    worst = _check_debug64(g, lt, S, P, oracle)
    print("configs4_all_64", gpu.last_fwd_bwd_kernel(), worst)


@pytest.mark.parametrize("flags", [F_TERM, 0, F_TERM | F_ZINF])
def test_debug64_ragged_and_edges(gpu, oracle, kernel_variant, flags):
    # infeasible (loss +inf / 0 with zero_infinity, every row -inf), single cell, S == P, log(0)
    # transitions, Z = 0, ragged lengths; the float64 state logs equal the oracle state's
    B, T, U = 9, 48, 33
    rng = np.random.default_rng(17)
    P = rng.integers(1, U + 1, size=B)
    S = np.array([rng.integers(max(1, p), T + 1) for p in P])
    S[0], P[0] = 1, 1
    S[1], P[1] = 10, 12
    S[2], P[2] = 0, 1
    S[3], P[3] = T, U
    S[4], P[4] = 20, 20
    lt = oracle.synth_log_trans(B, T, U, seed=17)
    lt[5, :, 3, 1] = -np.inf
    lt[6, :, :, :] = -np.inf  # Z = 0
    g = _run_debug64(gpu, lt, S, P, flags=flags)
    _check_debug64(g, lt, S, P, oracle, flags=flags)


def test_config5_long_form_bit_exact(gpu, oracle):
    # BASELINE configs[4] fwd-bwd: B=64 T=2000 U=400, bit-exact on every utterance, plus the
    # posterior-mass property
    B, T, U = 64, 2000, 400
    lt = oracle.synth_log_trans(B, T, U, seed=4)
    S, P = [T] * B, [U] * B
    g = _run_gpu(gpu, lt, S, P, debug=False)
    occ = -g["grad"][:, :T - 1].sum(axis=(2, 3))
    assert np.all(np.isfinite(g["loss"]))
    assert np.max(np.abs(occ - 1.0)) < 1e-3
    o = oracle.fwd_bwd_xf(lt, S, P)
    _assert_bit_exact(g, o, ["loss", "grad"])


@pytest.fixture(params=[pytest.param((1, 1), id="K1"), pytest.param((1, 0), id="K1-one-wg"),
                        pytest.param((2, 1), id="K2"), pytest.param((2, 0), id="K2-one-wg"),
                        pytest.param((1, 2), id="K1-split2", marks=pytest.mark.ab)])
def wide_lanes(request, gpu):
    """The long-row kernel's two lane widths (positions per lane), each with a direction's
    segments split over two workgroups (global hand-off) and in one workgroup, must be
    bit-identical."""
    k, split = request.param
    with gpu.use_ab() as ab:
        assert ab.ssnt_fwd_bwd_wide_lanes(k) == 0
        assert ab.ssnt_fwd_bwd_wide_split(split) == 0
        yield k
        ab.ssnt_fwd_bwd_wide_lanes(1)
        ab.ssnt_fwd_bwd_wide_split(-1)


WIDE_SHAPES = [  # the long-row kernel (256 < U <= 512): 3..8 waves per direction, odd U
    (2, 40, 257), (3, 33, 300), (2, 50, 383), (2, 41, 384), (3, 64, 400), (2, 29, 401), (2, 36, 512),
]


@pytest.mark.parametrize("shape", WIDE_SHAPES)
@pytest.mark.parametrize("obs", [False, True])
def test_wide_rows_bit_exact(gpu, oracle, wide_lanes, shape, obs):
    B, T, U = shape
    rng = np.random.default_rng(U + T)
    lt = oracle.synth_log_trans(B, T, U, seed=U)
    lo = (rng.standard_normal((B, T, U)) * 15 - 40).astype(np.float32) if obs else None
    P = [min(U, T)] + [int(x) for x in rng.integers(1, min(U, T) + 1, size=B - 1)]
    S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
    g = _run_gpu(gpu, lt, S, P, lo)
    o = oracle.fwd_bwd_xf(lt, S, P, log_obs=lo, debug=True)
    keys = ["loss", "grad", "log_alpha", "log_beta"] + (["grad_obs"] if obs else [])
    _assert_bit_exact(g, o, keys)


@pytest.mark.parametrize("flags", [F_TERM, 0, F_TERM | F_ZINF])
def test_wide_rows_edges(gpu, oracle, wide_lanes, flags):
    # single cell, S == P (one path), S < P (infeasible), S = 1, 2, 3 (cut at 0 / 1), a blocked
    # lattice (Z = 0), and lengths that end inside the first / last segment
    B, T, U = 10, 300, 300
    rng = np.random.default_rng(7)
    lt = oracle.synth_log_trans(B, T, U, seed=7)
    S = np.array([1, 280, 10, 1, 2, 3, 300, 300, 129, 257])
    P = np.array([1, 280, 12, 1, 2, 2, 300, 70, 128, 257])
    lt[7, :, :, 0] = -np.inf  # no emits and P < S: Z = 0
    lt[7, :, :, 1] = -np.inf
    g = _run_gpu(gpu, lt, S, P, flags=flags)
    o = oracle.fwd_bwd_xf(lt, S, P, flags=flags, debug=True)
    _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


def test_host_pointer_entry(gpu, oracle):
    from ssnt_tts_amd import capi
    lt = oracle.synth_log_trans(4, 30, 12, seed=1)
    lo = np.random.default_rng(1).standard_normal((4, 30, 12)).astype(np.float32)
    S, P = [30, 25, 12, 5], [12, 7, 12, 9]
    h = capi.ssnt_fwd_bwd(lt, S, P, log_obs=lo, debug=True)
    o = oracle.fwd_bwd_xf(lt, S, P, log_obs=lo, debug=True)
    _assert_bit_exact(h, o, ["loss", "grad", "grad_obs", "log_alpha", "log_beta"])


def test_autograd_function(gpu, oracle):
    dev = torch.device("cuda:0")
    lt = oracle.synth_log_trans(3, 20, 8, seed=4)
    x = torch.from_numpy(lt).to(dev).requires_grad_(True)
    S = torch.tensor([20, 15, 9], dtype=torch.int32, device=dev)
    P = torch.tensor([8, 8, 4], dtype=torch.int32, device=dev)
    loss = gpu.ssnt_lattice_loss(x, S, P)
    w = torch.tensor([1.0, 2.0, 0.5], device=dev)
    (loss * w).sum().backward()
    o = oracle.fwd_bwd_xf(lt, [20, 15, 9], [8, 8, 4])
    assert np.array_equal(loss.detach().cpu().numpy(), o["loss"])
    want = o["grad"] * np.array([1.0, 2.0, 0.5], np.float32)[:, None, None, None]
    assert np.array_equal(x.grad.cpu().numpy(), want)


def _wave_order_sum(loss):
    """The library's fixed summation order: 64 lane-strided f32 partial sums, then an xor
    butterfly (lattice_dev.h wave_loss_sum)."""
    acc = np.zeros(64, np.float32)
    for i, v in enumerate(np.asarray(loss, np.float32)):
        acc[i % 64] = np.float32(acc[i % 64] + v)
    off = 32
    while off >= 1:
        acc = (acc + acc[np.arange(64) ^ off]).astype(np.float32)
        off //= 2
    return acc[0]


@pytest.mark.parametrize("B", [1, 70, 256])
def test_fused_loss_sum(gpu, oracle, kernel_variant, B):
    # ssnt_fwd_bwd_sum_device: batch loss sum in the same launch (last workgroup), fixed order,
    # counter re-armed for the next call; infeasible utterances (+inf) included
    dev = torch.device("cuda:0")
    T, U = 40, 24
    rng = np.random.default_rng(B)
    lt = oracle.synth_log_trans(B, T, U, seed=B)
    P = rng.integers(1, U + 1, size=B)
    S = np.array([rng.integers(max(1, p), T + 1) for p in P])
    if B > 3:
        S[3], P[3] = 5, 9  # infeasible: loss 0 with zero_infinity
    o = oracle.fwd_bwd_xf(lt, S, P, flags=F_TERM | F_ZINF)
    want = _wave_order_sum(o["loss"])
    x = torch.from_numpy(lt).to(dev)
    sl = torch.tensor(S, dtype=torch.int32, device=dev)
    pl = torch.tensor(P, dtype=torch.int32, device=dev)
    for _ in range(3):  # the counter must re-arm itself between calls
        r = gpu.ssnt_fwd_bwd(x, sl, pl, zero_infinity=True, loss_sum=True, check=True)
        assert np.array_equal(r["loss"].cpu().numpy(), o["loss"])
        assert r["loss_sum"].cpu().numpy()[0] == want
    # without a counter: one extra single-wave pass, same bits
    lib = gpu.load()
    loss = torch.empty(B, device=dev)
    grad = torch.empty((B, T, U, 2), device=dev)
    lsum = torch.full((1,), -1.0, device=dev)
    import ctypes
    vp = ctypes.c_void_p
    wsb = int(lib.ssnt_fwd_bwd_workspace_size(B, T, U))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    rc = lib.ssnt_fwd_bwd_sum_device(vp(x.data_ptr()), None, vp(sl.data_ptr()), vp(pl.data_ptr()),
                                     B, T, U, F_TERM | F_ZINF, vp(loss.data_ptr()),
                                     vp(grad.data_ptr()), None, None, None, vp(ws.data_ptr()), wsb,
                                     None, vp(lsum.data_ptr()), None,
                                     vp(torch.cuda.current_stream(dev).cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    assert lsum.cpu().numpy()[0] == want


def test_fused_loss_sum_more_workgroups_than_cus(gpu, oracle, kernel_variant):
    # B = 2048 > 256 CUs: workgroup 0 waits for workgroups dispatched after it; the sum must still
    # be formed (and the state re-armed for the next call)
    dev = torch.device("cuda:0")
    B, T, U = 2048, 24, 16
    lt = oracle.synth_log_trans(B, T, U, seed=5)
    x = torch.from_numpy(lt).to(dev)
    sl = torch.full((B,), T, dtype=torch.int32, device=dev)
    pl = torch.full((B,), U, dtype=torch.int32, device=dev)
    o = oracle.fwd_bwd_xf(lt, [T] * B, [U] * B)
    for _ in range(2):
        r = gpu.ssnt_fwd_bwd(x, sl, pl, loss_sum=True, check=True)
        assert np.array_equal(r["loss"].cpu().numpy(), o["loss"])
        assert r["loss_sum"].cpu().numpy()[0] == _wave_order_sum(o["loss"])


@pytest.mark.parametrize("U", [79, 81, 127])
@pytest.mark.parametrize("obs", [False, True])
def test_lds_edge_rows_without_workspace_query_mismatch(gpu, oracle, U, obs):
    # T*U rows near the LDS budget with U % K != 0 (the narrow form pads rows) at T=200: the
    # workspace the library asks for must cover the kernel it then dispatches (with and without
    # log_obs, whose rings differ)
    B, T = 3, 200
    lt = oracle.synth_log_trans(B, T, U, seed=U)
    lo = (np.random.default_rng(U).standard_normal((B, T, U)) * 15 - 40).astype(np.float32) if obs else None
    S, P = [T, 150, 120], [U, U - 7, 40]
    g = _run_gpu(gpu, lt, S, P, lo, debug=False)
    o = oracle.fwd_bwd_xf(lt, S, P, log_obs=lo)
    _assert_bit_exact(g, o, ["loss", "grad"] + (["grad_obs"] if obs else []))


_C3 = {}


def _config4_oracle(oracle):
    """BASELINE configs[3] (B=2048 T=200 U=80, full lengths, seed 3): the oracle once per session."""
    if not _C3:
        B, T, U = 2048, 200, 80
        lt = oracle.synth_log_trans(B, T, U, seed=3)
        _C3.update(lt=lt, o=oracle.fwd_bwd_xf(lt, [T] * B, [U] * B))
    return _C3["lt"], _C3["o"]


def test_config4_global_batch_whole_and_sharded(gpu, oracle):
    # BASELINE configs[3]: B=2048 T=200 U=80, the global batch the 8-GPU run shards. On one GPU:
    # (1) the whole batch in one launch; (2) distributed.sharded_fwd_bwd over the 8 explicit
    # (rank, world=8) shards in sequence -- the exact slices each rank of the 8-GPU job runs.
    # Utterances are independent (src/lib.rs:122-133), so every shard is bit-exact against the
    # oracle's rows of the global batch, and the fused in-launch shard sum equals the library's
    # fixed-order sum of that shard.
    from ssnt_tts_amd.distributed import sharded_fwd_bwd, shard_bounds
    dev = torch.device("cuda:0")
    lt, o = _config4_oracle(oracle)
    B, T, U = lt.shape[:3]
    x = torch.from_numpy(lt).to(dev)
    sl = torch.full((B,), T, dtype=torch.int32, device=dev)
    pl = torch.full((B,), U, dtype=torch.int32, device=dev)
    r = gpu.ssnt_fwd_bwd(x, sl, pl, loss_sum=True, check=True)
    _assert_bit_exact({k: v.cpu().numpy() for k, v in r.items() if k in ("loss", "grad")}, o,
                      ["loss", "grad"])
    full_sum = r["loss_sum"].cpu().numpy()[0]
    assert full_sum == _wave_order_sum(o["loss"])
    del r
    shard_sums = []
    for rank in range(8):
        total, res, (lo, hi) = sharded_fwd_bwd(x, sl, pl, rank=rank, world=8, loss_sum=True,
                                               check=True)
        assert (lo, hi) == shard_bounds(B, 8, rank) and hi - lo == 256
        _assert_bit_exact({"loss": res["loss"].cpu().numpy(), "grad": res["grad"].cpu().numpy()},
                          {"loss": o["loss"][lo:hi], "grad": o["grad"][lo:hi]}, ["loss", "grad"])
        assert res["loss_sum"].cpu().numpy()[0] == _wave_order_sum(o["loss"][lo:hi])
        assert float(total) == float(res["loss_sum"].cpu().numpy()[0])  # (no process group: local)
        shard_sums.append(float(total))
    # the 8 ranks' all-reduce (a sum of 8 f32 shard sums) vs the one-launch global sum
    want = float(np.sum(o["loss"], dtype=np.float64))
    assert abs(sum(shard_sums) - want) <= 1e-5 * abs(want)
    assert abs(float(full_sum) - want) <= 1e-5 * abs(want)


@pytest.mark.parametrize("shape", [(2, 30, 700), (2, 24, 1024), (3, 26, 777)])
def test_rows_beyond_512_bit_exact(gpu, oracle, kernel_variant, shape):
    # 512 < U <= 1024: only the segmented kernel (two positions per lane, 8 waves per direction)
    # takes these; the two-wave kernel declines them
    if kernel_variant == 1:
        pytest.skip("the two-wave kernel stops at U = 512")
    B, T, U = shape
    rng = np.random.default_rng(U)
    lt = oracle.synth_log_trans(B, T, U, seed=U)
    P = [min(U, T)] + [int(x) for x in rng.integers(1, min(U, T) + 1, size=B - 1)]
    S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
    g = _run_gpu(gpu, lt, S, P)
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True)
    _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


@pytest.mark.parametrize("shift", [1, 2, 4])
@pytest.mark.parametrize("U", [80, 81, 127, 33])
def test_offset_and_odd_shapes(gpu, oracle, kernel_variant, shift, U):
    # log_trans AND grad at an element offset (4 / 8 / 16-byte aligned bases) and U % K != 0:
    # the streaming kernel's narrow form takes U % K != 0 and 4- or 8-byte alignment (one 8-byte
    # access per position), its vector form 16-byte alignment -- with identical bits
    dev = torch.device("cuda:0")
    B, T = 5, max(90, U + 10)
    lt = oracle.synth_log_trans(B, T, U, seed=shift + U)
    rng = np.random.default_rng(shift)
    P = [U] + [int(x) for x in rng.integers(1, U + 1, size=B - 1)]
    S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
    flat = torch.zeros(lt.size + shift, dtype=torch.float32, device=dev)
    flat[shift:] = torch.from_numpy(lt.ravel()).to(dev)
    x = flat[shift:].view(B, T, U, 2)
    assert x.data_ptr() % 16 == (4 * shift) % 16
    gflat = torch.full((lt.size + shift,), 7.0, dtype=torch.float32, device=dev)
    gv = gflat[shift:].view(B, T, U, 2)
    r = gpu.ssnt_fwd_bwd(x, torch.tensor(S, dtype=torch.int32, device=dev),
                         torch.tensor(P, dtype=torch.int32, device=dev), debug=True, check=True,
                         out={"grad": gv})
    if kernel_variant == 0 and shift % 4:  # the default dispatch keeps the streaming kernel
        assert gpu.last_fwd_bwd_kernel().startswith("k_fwd_bwd_stream<"), gpu.last_fwd_bwd_kernel()
        assert "NV=1" in gpu.last_fwd_bwd_kernel()
    g = {k: v.cpu().numpy() for k, v in r.items() if k != "status"}
    assert gflat[:shift].eq(7.0).all()  # nothing written before the view
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True)
    _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


LIVE_WIDE = [  # (B, T, U) with T >= U: every wave of the segmented kernel carries live positions
    (2, 1030, 1024),  # 2 positions per lane, 8 waves per direction
    (2, 920, 900),    # 2 per lane, 8 waves (last one partly live)
    (2, 520, 500),    # 1 per lane, 8 waves
    (3, 512, 480),    # 1 per lane, 8 waves (last one partly live)
]


@pytest.mark.parametrize("shape", LIVE_WIDE)
def test_rows_beyond_512_live_every_wave(gpu, oracle, kernel_variant, shape):
    # The segmented kernel's wave pipeline (5..8 waves per direction handing boundary values
    # through LDS) with live positions in every wave: utterance 0 spans the full U x T lattice,
    # the others are ragged with P past the first wave's 64K positions.
    if kernel_variant == 1 and shape[2] > 512:
        pytest.skip("the two-wave kernel stops at U = 512")
    B, T, U = shape
    rng = np.random.default_rng(T + U)
    lt = oracle.synth_log_trans(B, T, U, seed=T + U)
    P = [U] + [int(x) for x in rng.integers(U // 2, U + 1, size=B - 1)]
    S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
    g = _run_gpu(gpu, lt, S, P, debug=False)
    o = oracle.fwd_bwd_xf(lt, S, P)
    _assert_bit_exact(g, o, ["loss", "grad"])
    assert np.all(np.isfinite(g["loss"]))


@pytest.mark.parametrize("U", [500, 1000])
def test_rows_beyond_512_live_ragged_batch(gpu, oracle, wide_lanes, kernel_variant, U):
    # a ragged batch over the segmented kernel's range, both lane widths where U allows (one
    # position per lane stops at U = 512), debug rows too
    if kernel_variant == 1 and U > 512:
        pytest.skip("the two-wave kernel stops at U = 512")
    if wide_lanes == 1 and U > 512:
        pytest.skip("one position per lane stops at U = 512 (the K2 case covers it)")
    B, T = 6, U + 40
    lt = oracle.synth_log_trans(B, T, U, seed=11)
    P = np.array([U, U - 1, (2 * U) // 3, U // 2 + 13, 129, 1])
    S = np.array([T, U - 1, U - 50, (3 * U) // 4, T, 3])
    g = _run_gpu(gpu, lt, S, P)
    o = oracle.fwd_bwd_xf(lt, S, P, debug=True)
    _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


@pytest.mark.ab
@pytest.mark.parametrize("ring", [16, 32])
def test_stream_ring_depth_variants(gpu, oracle, kernel_variant, ring):
    # the streaming kernel's deeper-ring A/B form (16 / 32 factor slots, rows in the workspace)
    # must be bit-identical to the oracle (ragged batch, debug rows)
    if kernel_variant != 0:
        pytest.skip("a streaming-kernel form")
    with gpu.use_ab() as ab:
        assert ab.ssnt_fwd_bwd_stream_ring(ring) == 0
        rng = np.random.default_rng(ring)
        B, T, U = 6, 200, 80
        lt = oracle.synth_log_trans(B, T, U, seed=ring)
        P = [U] + [int(x) for x in rng.integers(1, U + 1, size=B - 1)]
        S = [T] + [int(rng.integers(p, T + 1)) for p in P[1:]]
        g = _run_gpu(gpu, lt, S, P)
        assert f"RS={ring}" in gpu.last_fwd_bwd_kernel() and "LDS=0" in gpu.last_fwd_bwd_kernel()
        o = oracle.fwd_bwd_xf(lt, S, P, debug=True)
        _assert_bit_exact(g, o, ["loss", "grad", "log_alpha", "log_beta"])


_TAG_SCRIPT = r"""
import ctypes, sys, torch
sys.path.insert(0, sys.argv[1])
import ssnt_tts_amd as S
import oracle as O
import numpy as np
lib = S.load()
lib.ssnt_diag_read.restype = ctypes.c_int
lib.ssnt_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert lib.ssnt_diag_read(None, 0) >= 0  # a diagnostic build (the product has no such symbol)
dev = torch.device("cuda:0")
for (B, T, U) in [(5, 90, 80), (256, 200, 80), (9, 48, 33), (4, 60, 65), (3, 45, 130)]:
    lt = O.synth_log_trans(B, T, U, seed=T + U)
    rng = np.random.default_rng(U)
    Pm = min(U, T)
    P = [Pm] + [int(x) for x in rng.integers(1, Pm + 1, size=B - 1)]
    Sl = [T] + [int(rng.integers(max(p, 1), T + 1)) for p in P[1:]]
    for debug in (False, True):
        r = S.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.tensor(Sl, dtype=torch.int32, device=dev),
                           torch.tensor(P, dtype=torch.int32, device=dev), debug=debug, check=False)
        bits = int(r["status"].item())
        assert bits == 0, (B, T, U, debug, bits, S.last_fwd_bwd_kernel())
        o = O.fwd_bwd_xf(lt, Sl, P)
        assert np.array_equal(r["loss"].cpu().numpy(), o["loss"]) and np.array_equal(r["grad"].cpu().numpy(), o["grad"])
print("ring tags ok")
"""


_TAG_FAULT_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import ssnt_tts_amd as S
import oracle as O
dev = torch.device("cuda:0")
for (B, T, U) in [(5, 90, 80), (4, 60, 80), (2, 40, 33), (2, 60, 64), (2, 70, 128), (3, 45, 130)]:
    lt = O.synth_log_trans(B, T, U, seed=1)
    Pm = min(T, U)
    r = S.ssnt_fwd_bwd(torch.from_numpy(lt).to(dev), torch.full((B,), T, dtype=torch.int32, device=dev),
                       torch.full((B,), Pm, dtype=torch.int32, device=dev), check=False)
    assert int(r["status"].item()) & 32, ("the tag check did not fire", B, T, U, S.last_fwd_bwd_kernel())
print("fault caught")
"""


def test_ring_tags_diag_build(kernel_variant):
    # the diagnostic build (make lib-diag) tags every converter-ring slot and
    # chain-ring row of the streaming kernel with the row it holds; every consumer checks the tag
    # after reading the data and sets kStatusRingTag on a mismatch. One process on that library:
    # configs[1], the B=5 T=90 U=80 case of the round-3 report, and the other lane layouts.
    import os
    import subprocess
    import sys
    from pathlib import Path
    if kernel_variant != 0:
        pytest.skip("the diagnostic library's own dispatch")
    root = Path(__file__).resolve().parent.parent
    lib = root / "ssnt-tts-rust_amd" / "lib" / "diag" / "libssnt_tts_c.so"
    assert lib.exists(), "make lib-diag"
    env = dict(os.environ, SSNT_TTS_C_LIB=str(lib), PYTHONPATH=str(root / "oracle"))
    r = subprocess.run([sys.executable, "-c", _TAG_SCRIPT, str(root / "ssnt-tts-rust_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ring tags ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    # negative control: the same build with converters that mislabel every slot (make
    # lib-diag-fault) must report the mismatch at every shape
    fault = root / "ssnt-tts-rust_amd" / "lib" / "diagfault" / "libssnt_tts_c.so"
    assert fault.exists(), "make lib-diag-fault"
    env["SSNT_TTS_C_LIB"] = str(fault)
    r = subprocess.run([sys.executable, "-c", _TAG_FAULT_SCRIPT, str(root / "ssnt-tts-rust_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "fault caught" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
