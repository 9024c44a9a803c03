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
