"""(r5) PodTopologySpread's weight is Go's math.Log(size + 2) (k8s v1.24.15 podtopologyspread/scoring.go
topologyNormalizingWeight), truncated after int64(cnt·w + maxSkew − 1).  The oracle (oracle/defaults.c or_go_log) and the
engine's host table (engine.hip go_log) restate Go's algorithm (src/math/log.go, the FreeBSD e_log.c reduction and
polynomial; amd64 evaluates the same expression without FMA).  This pins the restatement against an independent Python
transcription (Python floats are IEEE doubles with no contraction) over every size the engine can see, and records where
glibc's log() — what both sides used before r5 — differs, and whether any difference moves a PodTopologySpread score."""
import ctypes
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

LN2HI, LN2LO = 6.93147180369123816490e-01, 1.90821492927058770002e-10
L = (6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01, 2.222219843214978396e-01,
     1.818357216161805012e-01, 1.531383769920937332e-01, 1.479819860511658591e-01)
SQRT2_2 = 0.70710678118654752440


def go_log_py(x: float) -> float:
    """Transcription of Go's math.log for finite x > 0 (src/math/log.go)."""
    f1, ki = math.frexp(x)  # f1 in [0.5, 1), as Go's Frexp
    if f1 < SQRT2_2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L[0] + s4 * (L[2] + s4 * (L[4] + s4 * L[6])))
    t2 = s4 * (L[1] + s4 * (L[3] + s4 * L[5]))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * LN2HI - ((hfsq - (s * (hfsq + R) + k * LN2LO)) - f)


def _or_go_log():
    lib = O.lib()
    fn = lib.or_go_log
    fn.restype = ctypes.c_double
    fn.argtypes = [ctypes.c_double]
    return fn


def test_go_log_known_values():
    fn = _or_go_log()
    assert fn(1.0) == 0.0
    assert fn(2.0) == go_log_py(2.0) == 0.6931471805599453  # Go: math.Log(2) == Ln2
    assert math.isinf(fn(0.0)) and fn(0.0) < 0
    assert math.isnan(fn(-1.0))
    for x in (3.0, 10.0, 1e6 + 2, 2.0 ** 40, 1e-300):
        assert fn(x) == go_log_py(x)


def test_go_log_matches_transcription_over_all_sizes():
    """Every weight argument the engine tabulates: size + 2 for size in [0, 1M] (the node capacity bound is 2^19;
    zone counts are ≤ 64)."""
    fn = _or_go_log()
    bad = [f for f in range(0, 1_000_001) if fn(float(f + 2)) != go_log_py(float(f + 2))]
    assert bad == []


def test_go_log_vs_glibc_differences_and_their_effect():
    """Lists the sizes where glibc's log() differs from Go's (by at most one ulp), and checks whether the difference
    can move the PodTopologySpread raw score int64(cnt·w + maxSkew − 1) for counts up to 110 pods per node and
    maxSkew 1..5 — the figures DESIGN §3.15 quotes."""
    fn = _or_go_log()
    sizes = np.arange(0, 1_000_001, dtype=np.float64) + 2.0
    glibc = np.log(sizes)  # numpy's log is not glibc's either; take libm through ctypes for the record below
    libm = ctypes.CDLL("libm.so.6")
    libm.log.restype = ctypes.c_double
    libm.log.argtypes = [ctypes.c_double]
    diff = []
    for f in range(0, 1_000_001):
        x = float(f + 2)
        g, c = fn(x), libm.log(x)
        if g != c:
            assert abs(g - c) <= math.ulp(max(abs(g), abs(c)))
            diff.append(f)
    moved = []
    for f in diff:
        x = float(f + 2)
        g, c = fn(x), libm.log(x)
        for cnt in range(0, 111):
            for skew in range(1, 6):
                if int(cnt * g + skew - 1) != int(cnt * c + skew - 1):
                    moved.append((f, cnt, skew))
    out = os.environ.get("GO_LOG_REPORT")
    if out:
        with open(out, "w") as fh:
            fh.write(f"sizes where glibc log != Go log: {len(diff)} of 1000001\n")
            fh.write(f"first 50: {diff[:50]}\n")
            fh.write(f"(size, count, maxSkew) where the truncated raw score differs: {len(moved)}\n")
            fh.write(f"first 50: {moved[:50]}\n")
    assert len(glibc) == len(sizes)
