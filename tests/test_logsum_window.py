"""CPU check of the windowed exact sequential sum behind the GPU tonemapper (k_tm_winsum,
rtg_tonemap.hip): the same window rule restated in numpy -- inside one binade of the running
sum s, RN(s + x) = s + u * rint(x / u) with u = ulp(s); the first term that is a tie, leaves
the binade or meets s = 0 ends the window and takes one rounded add -- must give the reference's
left-to-right double sum (tonemapper.h:35-47) bit for bit.  The GPU kernel itself is checked
against the plain chain and the host sum in tests/test_gpu_tonemap.py."""
import math

import numpy as np
import pytest

WIN = 8192          # 8 waves x 64 lanes x 16 terms
LO, HI = 2 ** 52 + 1, 2 ** 53 - 2


def window_sum(x):
    n = len(x)
    s, a, fast = 0.0, 0, 0   # fast: terms that took the shortcut
    while a < n:
        win = x[a:a + WIN]
        fr, e = math.frexp(s)
        M = int(math.ldexp(fr, 53)) if s != 0.0 else 0
        y = np.ldexp(win, 53 - e)
        r = np.rint(y)
        ok = (s != 0.0) & (np.abs(y) < 2.0 ** 52) & (np.abs(y - r) != 0.5)
        k = np.where(ok, r, 0.0).astype(np.int64)
        P = M + np.cumsum(k)                       # running value after each term, units of u
        mag = -P if s < 0.0 else P
        bad = ~ok | (mag < LO) | (mag > HI)
        f = int(np.argmax(bad)) if bad.any() else len(win)
        fast += f
        if f > 0:
            s = math.ldexp(float(M + int(k[:f].sum())), e - 53)
        if f == len(win):
            a += len(win)
            continue
        s = s + float(win[f])                      # the stopping term: one rounded add
        if f < 64:                                 # slow region: the rest of the window as a chain
            for v in win[f + 1:].tolist():
                s = s + v
            a += len(win)
        else:
            a += f + 1
    return s, fast


def seq_sum(x):
    s = 0.0
    for v in x.tolist():
        s += v
    return s


def _logs(lum):
    return np.log(np.float64(np.float32(0.01)) + lum)


CASES = {
    "lognormal": lambda r: _logs(r.lognormal(0.0, 1.5, 300_000)),
    "bright": lambda r: _logs(r.lognormal(3.0, 1.0, 100_000)),
    "hover": lambda r: _logs(r.uniform(0.0, 1.98, 200_000)),
    "zero_logs": lambda r: np.zeros(50_000),
    "tiny_logs": lambda r: _logs(np.full(60_000, 0.99)),
    "black": lambda r: _logs(np.zeros(70_000)),
    "one": lambda r: _logs(np.array([2.0])),
    "ragged": lambda r: _logs(r.lognormal(0.0, 2.0, 8193)),
    "mixed_scale": lambda r: np.concatenate([r.normal(0, 1e-9, 20_000), r.normal(0, 50, 20_000),
                                             r.normal(3, 1e-3, 20_000)]),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_window_sum_equals_sequential(name):
    x = np.ascontiguousarray(CASES[name](np.random.default_rng(7)), np.float64)
    (got, fast), ref = window_sum(x), seq_sum(x)
    assert got == ref, (name, got.hex(), ref.hex())
    if name in ("lognormal", "bright", "black"):
        assert fast > 0.6 * len(x), (name, fast, len(x))   # the shortcut carries most of the sum


def summaries(x):
    """k_tm_wtot / k_tm_wguess / k_tm_wsumm: per aligned window, the guessed binade exponent at
    its start (from an approximate prefix of the window totals), the total Q of k = rint(x/u)
    and the least / greatest running partial, and whether the window is usable."""
    n = len(x)
    nw = (n + WIN - 1) // WIN
    tots = [float(np.sum(x[w * WIN:(w + 1) * WIN])) for w in range(nw)]
    out, s = [], 0.0
    for w in range(nw):
        e = math.frexp(s)[1] if s != 0.0 else None
        s += tots[w]
        win = x[w * WIN:(w + 1) * WIN]
        if e is None:
            out.append((None, 0, 0, 0, False))
            continue
        y = np.ldexp(win, 53 - e)
        r = np.rint(y)
        ok = (np.abs(y) < 2.0 ** 52) & (np.abs(y - r) != 0.5)
        k = np.where(ok, r, 0.0)
        usable = bool(ok.all()) and float(np.abs(k).sum()) < 2.0 ** 52
        P = np.cumsum(k.astype(np.int64))
        out.append((e, int(P[-1]), int(P.min()), int(P.max()), usable))
    return out


def summarised_sum(x):
    """k_tm_winsum<true>: windows end at aligned boundaries; an aligned window whose summary
    applies to the exact running sum is crossed in one step, every other takes the window rule."""
    n = len(x)
    summ = summaries(x)
    s, a, skipped = 0.0, 0, 0
    while a < n:
        if a % WIN == 0:
            e_g, Q, pmin, pmax, usable = summ[a // WIN]
            if usable and s != 0.0:
                fr, e = math.frexp(s)
                if e == e_g:
                    M = int(math.ldexp(fr, 53))
                    inside = (M + pmin >= LO and M + pmax <= HI) if s > 0 else (M + pmax <= -LO and M + pmin >= -HI)
                    if inside:
                        s = math.ldexp(float(M + Q), e - 53)
                        skipped += min(WIN, n - a)
                        a += WIN
                        continue
        lim = min(n, (a // WIN + 1) * WIN)
        win = x[a:lim]
        fr, e = math.frexp(s)
        M = int(math.ldexp(fr, 53)) if s != 0.0 else 0
        y = np.ldexp(win, 53 - e)
        r = np.rint(y)
        ok = (s != 0.0) & (np.abs(y) < 2.0 ** 52) & (np.abs(y - r) != 0.5)
        k = np.where(ok, r, 0.0).astype(np.int64)
        P = M + np.cumsum(k)
        mag = -P if s < 0.0 else P
        bad = ~ok | (mag < LO) | (mag > HI)
        f = int(np.argmax(bad)) if bad.any() else len(win)
        if f > 0:
            s = math.ldexp(float(M + int(k[:f].sum())), e - 53)
        if f == len(win):
            a = lim
            continue
        s = s + float(win[f])
        if f < 64:
            for v in win[f + 1:].tolist():
                s = s + v
            a = lim
        else:
            a += f + 1
    return s, skipped


@pytest.mark.parametrize("name", sorted(CASES))
def test_summarised_window_sum_equals_sequential(name):
    """Mode 3's rule (windows summarised in parallel, then crossed whole where the summary
    applies) gives the left-to-right double sum bit for bit."""
    x = np.ascontiguousarray(CASES[name](np.random.default_rng(7)), np.float64)
    (got, skipped), ref = summarised_sum(x), seq_sum(x)
    assert got == ref, (name, got.hex(), ref.hex())
    if name in ("bright", "black"):   # sums that run away from zero: most windows crossed whole
        assert skipped > 0.5 * len(x), (name, skipped, len(x))
