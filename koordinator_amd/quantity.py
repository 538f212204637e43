"""k8s resource.Quantity parsing (subset) into the engine's integer units.

`resource.MustParse` strings ("16", "500m", "32Gi", "1.5") → exact integers.  The engine stores cpu in
milli-units (Quantity.MilliValue) and everything else in Quantity.Value, both rounded up like apimachinery
(k8s.io/apimachinery v0.24 resource.Quantity.MilliValue/Value use ceil for fractional results).
"""
from __future__ import annotations

from fractions import Fraction

_BINARY = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DECIMAL = {"n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": Fraction(1),
            "k": Fraction(10**3), "M": Fraction(10**6), "G": Fraction(10**9), "T": Fraction(10**12),
            "P": Fraction(10**15), "E": Fraction(10**18)}


def parse(q) -> Fraction:
    """Exact value of a quantity string (or number)."""
    if isinstance(q, (int, Fraction)):
        return Fraction(q)
    if isinstance(q, float):
        return Fraction(str(q))
    s = str(q).strip()
    for suf, mul in _BINARY.items():
        if s.endswith(suf):
            return Fraction(s[: -len(suf)]) * mul
    if s and s[-1] in "numkMGTPE" and not s[-1].isdigit():
        return Fraction(s[:-1]) * _DECIMAL[s[-1]]
    if "e" in s.lower():
        return Fraction(s)
    return Fraction(s)


def _ceil(f: Fraction) -> int:
    return -((-f.numerator) // f.denominator)


def milli_value(q) -> int:
    return _ceil(parse(q) * 1000)


def value(q) -> int:
    return _ceil(parse(q))


def resource_value(name: str, q) -> int:
    """getResourceValue (pkg/scheduler/plugins/loadaware/helper.go:146-151): cpu → MilliValue, else Value."""
    return milli_value(q) if name == "cpu" else value(q)
