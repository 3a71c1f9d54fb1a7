"""CPU models of the wave-walk algorithms of walk.hip (no GPU): each model
follows the kernel's decomposition -- LeapCDC's per-word orbit tables built by
the forward "last failing window" pass and the backward result pass, the
512-position block tables chased through 8 word tables (jtab_kernel), and
wcut_leap's walk over them; SeqCDC's 4096-position
windows with the carried run / opposing-pair count and the restarts a jump
lands inside the window (wcut_seq); UltraCDC's 512-block windows with the
LEST run carried between windows (wcut_ultra) -- and must reproduce the
oracle's byte rules (oracle/cdc_oracle.c cut_leap / cut_seq / cut_ultra)
chunk for chunk.  The GPU kernels themselves are checked against the oracle
by tests/test_gpu_walk.py and tests/test_gpu_configs.py.
"""
import numpy as np
import pytest

import oracle

P = oracle._cdc_params()
M64 = (1 << 64) - 1


# ---- LeapCDC ----------------------------------------------------------------

def leap_bitmaps(d, mn, avg):
    """Primary / secondary eligibility of the 5-byte window ending at each
    position (bits_kernel<5>); positions < 4 are never tested (min >= 32)."""
    E = np.array([oracle._mix64((P["CDC_LEAP_SEED"] + (b + 1) * 0x9E3779B97F4A7C15) & M64)
                  for b in range(256)], dtype=np.uint64)
    thr = P["THR"][min(oracle._log2_round(max(avg - mn, 1)), 32)]
    n = d.size
    h = np.zeros(n, dtype=np.uint64)
    e = E[d]
    with np.errstate(over="ignore"):
        for j in range(P["CDC_LEAP_WSIZE"]):
            r = np.uint64((11 * j) % 64)
            rot = (e << r) | (e >> (np.uint64(64) - r)) if r else e
            h[j:] += rot[:n - j]
    prim = (h >> np.uint64(32)) < thr
    sec = (h & np.uint64(0xFFFFFFFF)) < thr
    return prim, sec


def leap_tables(prim, sec):
    """jtab_kernel: per 64-position word, the orbit result of entries 0..23
    (< 24: entry into the next word, >= 64: accepted at offset v - 64)."""
    n = prim.size
    nw = (n + 63) // 64
    pad = np.zeros(nw * 64 + 64, dtype=bool)
    sp = pad.copy()
    pad[64:64 + n] = prim   # index i + 64 <-> position i (64 words of zero pad before)
    sp[64:64 + n] = sec
    WIN, PRI = P["CDC_LEAP_WINDOWS"], P["CDC_LEAP_PRIMARY"]
    tabs = np.zeros((nw, 24), dtype=np.int64)
    for w in range(nw):
        b = 64 * w + 64  # pad index of the word's position 0
        fail = ~pad[b - 64:b + 64]  # positions 64w-64 .. 64w+63
        lo = np.nonzero(fail[:64])[0]
        lz = (int(lo[-1]) - 64) if lo.size else -1000
        nxt = [0] * 64
        for x in range(64):
            if x > 0 and fail[64 + x - 1]:
                lz = x - 1
            if lz >= x - PRI:
                nxt[x] = lz + WIN + 1
            elif not sp[b + x - PRI - 1]:
                nxt[x] = x + 2
            elif not sp[b + x - PRI - 2]:
                nxt[x] = x + 1
            else:
                nxt[x] = 255
        res = [0] * 64
        for x in range(63, -1, -1):
            v = nxt[x]
            res[x] = 64 + x if v == 255 else v - 64 if v >= 64 else res[v]
        tabs[w] = res[:24]
    return tabs


def leap_step(prim, sec, c):
    """cut_leap_bits' leap at candidate c: 0 = accepted."""
    WIN, PRI = P["CDC_LEAP_WINDOWS"], P["CDC_LEAP_PRIMARY"]
    f = prim[c - PRI:c]
    z = np.nonzero(~f)[0]
    if z.size:
        return WIN - (PRI - 1 - int(z[-1]))
    if not sec[c - PRI - 1]:
        return WIN - PRI
    if not sec[c - PRI - 2]:
        return WIN - PRI - 1
    return 0


def block_tables(tabs):
    """The 512-position block tables: each entry chased through 8 word tables
    (< 24: entry into the next block, >= 512: accepted at offset v - 512)."""
    nb = (tabs.shape[0] + 7) // 8
    t8 = np.zeros((nb, 24), dtype=np.int64)
    for b in range(nb):
        for e in range(24):
            x, v = e, None
            for t in range(8):
                if 8 * b + t >= tabs.shape[0]:
                    break
                u = int(tabs[8 * b + t, x])
                if u >= 64:
                    v = 512 + 64 * t + (u - 64)
                    break
                x = u
            t8[b, e] = x if v is None else v
    return t8


def wcut_leap(prim, sec, tabs, t8, s, n, mn, mx):
    """wcut_leap: leaps in the start candidate's word, then word tables to the
    next block boundary, block tables while a whole block is <= E, word tables
    up to E's word (acceptance past E = no content-defined cut)."""
    if n <= mn:
        return n
    end = min(n, mx)
    E = s + end
    c = s + mn
    w = c >> 6
    while c < 64 * (w + 1):
        if c > E:
            return end
        lp = leap_step(prim, sec, c)
        if not lp:
            return c - s
        c += lp
    w, e = w + 1, c & 63
    while True:
        if 64 * w + e > E:
            return end
        if w % 8 == 0 and 64 * (w + 8) - 1 <= E:
            v = int(t8[w // 8, e])
            if v >= 512:
                return 64 * w + (v - 512) - s
            e, w = v, w + 8
            continue
        v = int(tabs[w, e])
        if v >= 64:
            pos = 64 * w + (v - 64)
            return pos - s if pos <= E else end
        e, w = v, w + 1


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (512, 2048, 16384), (2048, 8192, 65536)])
def test_leap_word_tables_model(sizes):
    mn, avg, mx = sizes
    d = oracle.splitmix64_bytes((1 << 20) + 777, 5)
    prim, sec = leap_bitmaps(d, mn, avg)
    tabs = leap_tables(prim, sec)
    t8 = block_tables(tabs)
    got, pos = [], 0
    while pos < d.size:
        cut = wcut_leap(prim, sec, tabs, t8, pos, d.size - pos, mn, mx)
        got.append((pos, cut))
        pos += cut
    ref = oracle.cdc("leap", d, mn, avg, mx)
    assert np.array_equal(np.array(got, dtype=np.uint64).reshape(-1, 2), ref)


# ---- SeqCDC -----------------------------------------------------------------

def wcut_seq(y, s, n, mn, mx, L, T, J, win=4096):
    """wcut_seq: windows of `win` pair bits; from each restart t0 the first
    completed run of L in-direction pairs (the run carried into the window
    counts when t0 = 0) against the (T - opp)-th opposing pair at or after t0."""
    if n <= mn:
        return n
    end = min(n, mx)
    i, cnt, opp = mn, 0, 0
    while i < end:
        lim = end - i
        k = min(win, lim)
        yy = y[s + i:s + i + k]
        t0, opp0, carried = 0, opp, True
        while True:
            # run event
            tr = None
            run = cnt if carried else 0
            for t in range(t0, k):
                run = run + 1 if yy[t] else 0
                if run >= L:
                    tr = t
                    break
            # jump event
            zs = np.nonzero(~yy[t0:])[0]
            need = T - opp0
            tj = t0 + int(zs[need - 1]) if zs.size >= need else None
            if tr is not None and (tj is None or tr < tj):
                return i + tr + 1
            if tj is None:
                if lim <= win:
                    return end
                r = 0
                for t in range(win - 1, t0 - 1, -1):
                    if not yy[t]:
                        break
                    r += 1
                cnt = r if not (carried and r == win) else cnt + r
                opp = opp0 + int(zs.size)
                i += win
                break
            t0, opp0, carried = tj + J, 0, False
            if t0 >= win or t0 >= lim:
                i += t0
                cnt = opp = 0
                break
    return end


@pytest.mark.parametrize("data", ["random", "periodic", "runs"])
def test_seq_window_events_model(data):
    mn, avg, mx = 4096, 8192, 16384
    L, T, J = P["CDC_SEQ_LENGTH"], P["CDC_SEQ_JUMP_TRIGGER"], P["CDC_SEQ_JUMP_SIZE"]
    n = (1 << 19) + 333
    if data == "random":
        d = oracle.splitmix64_bytes(n, 11)
    elif data == "periodic":
        d = np.resize(oracle.splitmix64_bytes(61, 7), n)
    else:  # long increasing runs: run events and carried runs across windows
        d = (np.arange(n) % 251).astype(np.uint8)
    y = np.zeros(n, dtype=bool)
    y[1:] = d[1:] > d[:-1]  # increasing mode
    got, pos = [], 0
    while pos < n:
        cut = wcut_seq(y, pos, n - pos, mn, mx, L, T, J)
        got.append((pos, cut))
        pos += cut
    ref = oracle.cdc("seq", d, mn, avg, mx)
    assert np.array_equal(np.array(got, dtype=np.uint64).reshape(-1, 2), ref)


# ---- UltraCDC ---------------------------------------------------------------

def ultra_bitmaps(d):
    n = d.size
    pat = P["CDC_ULTRA_PATTERN"]
    c = np.array([bin(b ^ pat).count("1") for b in range(256)], dtype=np.int64)[d]
    cs = np.concatenate([[0], np.cumsum(c)])
    dist = np.zeros(n, dtype=np.int64)
    dist[8:] = cs[8:n] - cs[0:n - 8]  # bytes q-8 .. q-1
    hs = (dist & P["CDC_ULTRA_MASK_S"]) == 0
    hl = (dist & P["CDC_ULTRA_MASK_L"]) == 0
    eqb = np.zeros(n, dtype=bool)
    eqb[8:] = d[8:] == d[:-8]
    rep = np.zeros(n, dtype=bool)  # bytes q..q+7 equal the 8 before
    ok = np.ones(max(n - 7, 0), dtype=bool)
    for t in range(8):
        ok &= eqb[t:n - 7 + t]
    rep[:n - 7] = ok
    return hs, hl, rep


def wcut_ultra(hs, hl, rep, s, n, mn, avg, mx, LEST, wblk=512):
    if n <= mn:
        return n
    normal, end = avg, n
    if n >= mx:
        end = mx
    elif n <= normal:
        normal = n
    if end < mn + 8:
        return end
    nblk = (end - mn) >> 3
    tnorm = (normal - mn + 7) >> 3 if normal > mn else 0
    lec = 0
    for t0 in range(0, nblk, wblk):  # one window of blocks per step
        for t in range(t0, min(t0 + wblk, nblk)):
            q = s + mn + 8 * t
            if rep[q]:
                lec += 1
                if lec >= LEST:
                    return mn + 8 * t + 8
                continue
            lec = 0
            h = hs if t < tnorm else hl
            hit = np.nonzero(h[q:q + 8])[0]
            if hit.size:
                return mn + 8 * t + int(hit[0])
    return end


@pytest.mark.parametrize("data", ["random", "zeros", "mixed"])
def test_ultra_block_windows_model(data):
    mn, avg, mx = 4096, 8192, 16384
    n = (1 << 19) + 1001
    if data == "random":
        d = oracle.splitmix64_bytes(n, 3)
    elif data == "zeros":
        d = np.zeros(n, dtype=np.uint8)
    else:
        d = oracle.splitmix64_bytes(n, 4)
        d[100000:300013] = 0
    hs, hl, rep = ultra_bitmaps(d)
    got, pos = [], 0
    while pos < n:
        cut = wcut_ultra(hs, hl, rep, pos, n - pos, mn, avg, mx, P["CDC_ULTRA_LEST"])
        got.append((pos, cut))
        pos += cut
    ref = oracle.cdc("ultra", d, mn, avg, mx)
    assert np.array_equal(np.array(got, dtype=np.uint64).reshape(-1, 2), ref)


def ultra_run(rep, c, n, lim, mn, mx, LEST):
    """walk.hip ultra_run: LEST chunks the chain takes at once from c inside a
    run of 8-byte repeats (starts < lim), from the first non-repeat position
    at or after c + min."""
    Lr = mn + 8 * LEST
    if mx < Lr or c >= lim or n - c < Lr:
        return 0
    kmax = min((n - c) // Lr, (lim - c + Lr - 1) // Lr)
    a, tail = c + mn, 8 * LEST - 8
    need = a + (kmax - 1) * Lr + tail + 1
    z = np.nonzero(~rep[a:need])[0]
    b = a + int(z[0]) if z.size else need
    return min(kmax, (b - a - tail + Lr - 1) // Lr) if b > a + tail else 0


def repeat_regions(n, seed):
    d = oracle.splitmix64_bytes(n, seed)
    d[10007:10007 + 300000] = 0                                   # zeros, unaligned
    d[400001:400001 + 123457] = 0x41                              # a constant byte
    d[600003:600003 + 250000] = np.resize(np.arange(8, dtype=np.uint8) * 37, 250000)  # 8-byte period
    d[900000:900000 + 70000] = 0
    d[900000 + 33333] = 1                                         # one break inside a zero run
    return d


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (512, 2048, 16384), (2048, 8192, 65536)])
def test_ultra_repeat_runs_model(sizes):
    """Chains that take a repeat run's LEST chunks many at a time (ultra_run
    after a chunk of exactly min + 8 LEST) cut exactly where the oracle does."""
    mn, avg, mx = sizes
    LEST = P["CDC_ULTRA_LEST"]
    Lr = mn + 8 * LEST
    n = (1 << 20) + 4321
    d = repeat_regions(n, 9)
    hs, hl, rep = ultra_bitmaps(d)
    got, pos, jumped = [], 0, 0
    while pos < n:
        cut = wcut_ultra(hs, hl, rep, pos, n - pos, mn, avg, mx, LEST)
        got.append((pos, cut))
        pos += cut
        if cut == Lr:
            k = ultra_run(rep, pos, n, n, mn, mx, LEST)
            got += [(pos + j * Lr, Lr) for j in range(k)]
            pos += k * Lr
            jumped += k
    ref = oracle.cdc("ultra", d, mn, avg, mx)
    assert np.array_equal(np.array(got, dtype=np.uint64).reshape(-1, 2), ref)
    if mx >= Lr:
        assert jumped > 0


def quiet_run(loud, c, n, lim, L, lo, hi):
    """walk.hip quiet_run over a boolean 'loud' array (generic form of ultra_run)."""
    if c >= lim or n - c < L:
        return 0
    kmax = min((n - c) // L, (lim - c + L - 1) // L)
    a, tail = c + lo, hi - lo
    need = a + (kmax - 1) * L + tail + 1
    z = np.nonzero(loud[a:need])[0]
    b = a + int(z[0]) if z.size else need
    return min(kmax, (b - a - tail + L - 1) // L) if b > a + tail else 0


def walk_with_quiet_runs(cut, loud, n, L, lo, hi):
    """The wave walks' loop: after two chunks of exactly L in a row, take the
    quiet run's chunks at once (take_run)."""
    got, pos, pq, jumped = [], 0, False, 0
    while pos < n:
        d = cut(pos)
        got.append((pos, d))
        pos += d
        q = d == L
        if q and pq:
            k = quiet_run(loud, pos, n, n, L, lo, hi)
            got += [(pos + j * L, L) for j in range(k)]
            pos += k * L
            jumped += k
            pq = k != 0
        else:
            pq = q
    return np.array(got, dtype=np.uint64).reshape(-1, 2), jumped


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (2048, 8192, 65536)])
def test_quiet_runs_model_seq_leap(sizes):
    """SeqCDC (L = max over pair-free runs) and LeapCDC (L = min over
    all-eligible runs) with quiet-run jumps cut exactly where the oracle does
    on zero-filled / constant regions at unaligned offsets."""
    mn, avg, mx = sizes
    n = (1 << 20) + 4321
    d = repeat_regions(n, 21)
    # SeqCDC, increasing mode
    Ls, Ts, Js = P["CDC_SEQ_LENGTH"], P["CDC_SEQ_JUMP_TRIGGER"], P["CDC_SEQ_JUMP_SIZE"]
    y = np.zeros(n, dtype=bool)
    y[1:] = d[1:] > d[:-1]
    got, jumped = walk_with_quiet_runs(lambda s: wcut_seq(y, s, n - s, mn, mx, Ls, Ts, Js), y, n, mx, mn - 1, mx - 1)
    assert np.array_equal(got, oracle.cdc("seq", d, mn, avg, mx))
    assert jumped > 0
    # LeapCDC
    prim, sec = leap_bitmaps(d, mn, avg)
    tabs = leap_tables(prim, sec)
    t8 = block_tables(tabs)
    W = P["CDC_LEAP_WINDOWS"]
    loud = ~(prim & sec)
    got, jumped = walk_with_quiet_runs(lambda s: wcut_leap(prim, sec, tabs, t8, s, n - s, mn, mx), loud, n, mn,
                                       mn - W, mn - 1)
    assert np.array_equal(got, oracle.cdc("leap", d, mn, avg, mx))
