#!/usr/bin/env python3
"""Integer restatement of the reference's double-precision bit scans (KProcessor.java:371-377).

    getFirstSetBitPos(n) = (int)(Math.log10(n & -n) / Math.log10(2))
    getLastSetBitPos(n)  = (int)(Math.log10((double) n) / Math.log10(2))

With a correctly rounded log10 (HotSpot's Math.log10 is specified within 1 ulp; the value at
these points is pinned here under correct rounding, parity unpinned against a real JVM):
  * first(): exact ctz for every power of two 2^0..2^62 (2^63 is negative -> NaN -> 0);
  * last(): h = 63 - clz(n), except that it returns h + 1 once n >= T[h] = 2^(h+1) - D[h], h >= 47.

Prints D[47..62] (the table in oracle/kme_oracle.c and kme_kernels.hip) and, with --glibc, the
thresholds glibc's log10 would give instead.
"""
import math
import sys
from decimal import Decimal, getcontext

getcontext().prec = 80


def cr_log10(x: float) -> float:
    return float(Decimal(x).log10())


def quotient_cr(n: int) -> int:
    return int(cr_log10(float(n)) / cr_log10(2.0))


def quotient_glibc(n: int) -> int:
    return int(math.log10(float(n)) / math.log10(2))


def thresholds(f):
    D = {}
    for h in range(63):
        lo, hi = 2 ** h, 2 ** (h + 1) - 1
        assert f(lo) >= h
        if f(hi) <= h:
            continue
        a, b = lo, hi
        while a < b:
            m = (a + b) // 2
            if f(m) >= h + 1:
                b = m
            else:
                a = m + 1
        D[h] = 2 ** (h + 1) - a
    return D


def first_exact() -> bool:
    return all(int(cr_log10(float(2 ** k)) / cr_log10(2.0)) == k for k in range(63))


if __name__ == "__main__":
    assert first_exact()
    D = thresholds(quotient_cr)
    print("correctly rounded log10: D[h] for h =", min(D), "..", max(D))
    print(", ".join(str(D[h]) for h in sorted(D)))
    if "--glibc" in sys.argv:
        G = thresholds(quotient_glibc)
        print("glibc log10:", ", ".join(str(G[h]) for h in sorted(G)))
