#!/usr/bin/env python3
"""Double-double coefficient tables of vo_crmath.h (division-free series): prints C array
initialisers (hi, lo pairs, hex floats) computed with 300-bit mpmath.  hi = RN(c), lo =
RN(c - hi).  Usage: python tools/gen_crmath_tables.py > /tmp/tables.h"""
import mpmath

mpmath.mp.prec = 300


def dd(c):
    hi = float(c)
    lo = float(c - mpmath.mpf(hi))
    return hi, lo


def table(name, vals):
    print(f"VCR_TAB double {name}[{2 * len(vals)}] = {{")
    for v in vals:
        hi, lo = dd(v)
        print(f"    {hi.hex()}, {lo.hex()},")
    print("};")


one = mpmath.mpf(1)
# sin / cos nested Taylor: index k (1..31): 1/((2k)(2k+1)) and 1/((2k-1)(2k))
table("VCR_SIN_C", [one / ((2 * k) * (2 * k + 1)) if k else one for k in range(0, 32)])
table("VCR_COS_C", [one / ((2 * k - 1) * (2 * k)) if k else one for k in range(0, 32)])
# asin nested series: (2k-1)^2 / ((2k)(2k+1)), k = 0..60
table("VCR_ASIN_C", [mpmath.mpf((2 * k - 1) ** 2) / ((2 * k) * (2 * k + 1)) if k else one for k in range(0, 61)])
# exp nested Taylor: 1/k, k = 0..24
table("VCR_EXP_C", [one / k if k else one for k in range(0, 25)])
# log atanh series: (2k-1)/(2k+1), k = 0..22
table("VCR_LOG_C", [mpmath.mpf(2 * k - 1) / (2 * k + 1) if k else one for k in range(0, 23)])
