"""Independent pure-Python restatement of the reference decode steps -- TEST INFRASTRUCTURE.

Written separately from oracle/ssnt_oracle.c (different language, different structure: Python's
stable `sorted`, explicit usize arithmetic mod 2^64) so that the two restatements cross-check
each other on random and tie-rich inputs. Small cases only.
Cites: src/lib.rs:149-230 (v1), src/v2.rs:94-339 (v2), src/tone_latent.rs:184-234 (tone).
"""
import numpy as np

M64 = 1 << 64


def usize(v):
    return int(v) % M64  # Rust `i32 as usize` (sign extension) for |v| < 2^63


def i32(v):
    v = int(v) % (1 << 32)
    return v - (1 << 32) if v >= (1 << 31) else v


def f32add(a, b):
    return np.float32(np.float32(a) + np.float32(b))


def _merge(cands, Wmax, keys):
    # stable sort by log_prob descending (src/lib.rs:161), then consecutive dedup (:162)
    order = sorted(range(len(cands)), key=lambda i: -float(cands[i]["lp"]))
    s = [cands[i] for i in order]
    out = []
    for c in s:
        if out and all(c[k] == out[-1][k] for k in keys):
            continue
        out.append(c)
    return out


def _pack(res, with_tot=False):
    d = dict(prediction=np.array([r["pred"] for r in res], np.int32),
             log_prob=np.array([r["lp"] for r in res], np.float32),
             next_t=np.array([i32(r["nt"]) for r in res], np.int32),
             next_u=np.array([i32(r["nu"]) for r in res], np.int32),
             next_is_finished=np.array([r["fin"] for r in res], bool),
             beam_branch=np.array([r["parent"] for r in res], np.int32))
    if with_tot:
        d["next_total_duration"] = np.array([r["tot"] for r in res], np.int32)
    return d


def v1_step(h, hist, fin, t, u, input_length, Wmax):
    W = len(hist)
    I = usize(input_length)
    cands = []
    for w in range(W):
        tw, uw = usize(t[w]), usize(u[w])
        if not (tw < I) or fin[w]:
            cands.append(dict(pred=0, lp=np.float32(hist[w]), nt=tw, nu=uw, fin=True, parent=w))
            continue
        last = (I - 1) % M64
        for k in (0, 1):
            v = h[w][k]
            if k == 0 and tw == last:
                c = dict(pred=0, lp=f32add(hist[w], v), nt=tw, nu=uw, fin=True)
            elif k == 1 and tw == last:
                c = dict(pred=0, lp=np.float32(hist[w]), nt=tw, nu=uw, fin=True)
            elif k == 1:
                c = dict(pred=1, lp=f32add(hist[w], v), nt=(tw + 1) % M64, nu=(uw + 1) % M64, fin=False)
            else:
                c = dict(pred=0, lp=f32add(hist[w], v), nt=tw, nu=(uw + 1) % M64, fin=False)
            c["parent"] = w
            cands.append(c)
    kept = _merge(cands, Wmax, ("pred", "lp", "nt", "nu", "fin"))
    res = [kept[i % len(kept)] for i in range(Wmax)]
    return _pack(res)


def _f2i(x):
    x = np.float32(x)
    if np.isnan(x):
        return 0
    if x >= 2147483648.0:
        return 2147483647
    if x <= -2147483648.0:
        return -2147483648
    return int(x)  # truncation toward zero


def v2_step(h, hist, fin, total, table, t, u, input_length, output_length, zid, allow_skip,
            test_mode, Wmax):
    W, D = h.shape
    I, O = usize(input_length), usize(output_length)
    fO, fI = np.float32(O), np.float32(I)

    def bounds(tt):
        diag = np.float32(np.float32(fO / fI) * np.float32(tt + 1))
        up = np.float32(fO * np.float32(0.1))
        lo = np.float32(fO * np.float32(0.05))
        return _f2i(max(np.float32(diag - lo), np.float32(0.0))), _f2i(min(np.float32(diag + up), fO))

    cands = []
    for w in range(W):
        tw, uw = usize(t[w]), usize(u[w])
        if not (tw < I) or fin[w]:
            cands.append(dict(pred=zid, lp=np.float32(hist[w]), nt=tw, nu=uw, fin=True, parent=w,
                              tot=int(total[w])))
            continue
        lb, ub = bounds(tw)
        overrun = ((I - (tw + 1)) * 3) % M64 > O
        for i in range(D):
            tot = i32(int(total[w]) + int(table[i]))
            if not test_mode and (tot < lb or tot > ub):
                continue
            if not test_mode and overrun:
                continue
            if tw == (I - 1) % M64:
                if not test_mode and tot != i32(O):
                    continue
                if not allow_skip and i == zid:
                    continue
                isfin = True
            else:
                if not allow_skip and i == zid:
                    continue
                isfin = False
            cands.append(dict(pred=i, lp=f32add(hist[w], h[w][i]), nt=tw if isfin else (tw + 1) % M64,
                              nu=uw if isfin else (uw + 1) % M64, fin=isfin, parent=w, tot=tot))
    kept = _merge(cands, Wmax, ("pred", "lp", "nt", "nu", "fin", "tot"))
    if not kept:
        return None
    diag = None
    if not test_mode:
        for c in kept:
            d = np.float32(np.float32(fO / fI) * np.float32(c["nt"]))
            diff = np.float32(np.float32(c["tot"]) - d)
            if -20.0 <= diff <= 0.0:
                diag = c
                break
    res = [kept[i % len(kept)] for i in range(Wmax)]
    if diag is not None:
        res = res[:Wmax - 1] + [diag]
    return _pack(res, with_tot=True)


def tone_step(h, hist, fin, t, u, input_length, empty_id, Wmax):
    W, C = h.shape
    I = usize(input_length)
    cands = []
    for w in range(W):
        tw, uw = usize(t[w]), usize(u[w])
        if not (tw < I) or fin[w]:
            cands.append(dict(pred=empty_id, lp=np.float32(hist[w]), nt=tw, nu=uw, fin=True, parent=w))
            continue
        for i in range(C):
            cands.append(dict(pred=i, lp=f32add(hist[w], h[w][i]), nt=(tw + 1) % M64,
                              nu=(uw + 1) % M64, fin=False, parent=w))
    kept = _merge(cands, Wmax, ("pred", "lp", "nt", "nu", "fin"))
    res = [kept[i % len(kept)] for i in range(Wmax)]
    return _pack(res)
