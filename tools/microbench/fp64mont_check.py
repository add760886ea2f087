#!/usr/bin/env python3
"""Checks tools/microbench/fp64mont.hip's dump: every line holds a, b and
out = mont52(mont52(a, b), b) as 52-bit hex limbs; out must be congruent to
a b^2 R^-2 mod p (R = 2^260) and below 2p."""
import sys

P = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47
RI = pow(1 << 260, -1, P)


def val(field):
    return sum(int(x, 16) << (52 * i) for i, x in enumerate(field.split(",")))


bad = n = 0
for line in open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/fp64mont_dump.txt"):
    a, b, out = (val(f) for f in line.split())
    n += 1
    if out >= 2 * P or (out - a * b * b * RI * RI) % P:
        bad += 1
print(f"fp64mont: {n - bad}/{n} products correct")
sys.exit(1 if bad or not n else 0)
