"""Exact check of the Muon kernel's normalisation quotient (optim.hip, muon_kernel): for a uniform
divisor d, q0 = RN(y * RN(1/d)), e = RN(y - q0 d) (fma), q = RN(q0 + e RN(1/d)) (fma) equals the
correctly rounded fp32 y / d for every pair of bf16 significands (rational arithmetic; the result is
independent of the exponents in the normal range).   python tools/check_bf16_division.py"""
from fractions import Fraction as F
import math
def rn32(x):
    # round a Fraction to nearest float32 (ties to even), normal range assumed
    if x == 0: return F(0)
    s = -1 if x < 0 else 1; x = abs(x)
    e = math.floor(math.log2(x.numerator) - math.log2(x.denominator))
    # adjust e so that 2^e <= x < 2^(e+1)
    while F(2)**e > x: e -= 1
    while F(2)**(e+1) <= x: e += 1
    ulp = F(2)**(e-23)
    q = x / ulp
    n = q.numerator // q.denominator
    r = q - n
    if r > F(1,2) or (r == F(1,2) and n % 2 == 1): n += 1
    return s * n * ulp
bad = 0
for my in range(128, 256):
    y = F(my, 128)
    for mn in range(128, 256):
        d = F(mn, 128) * 8   # nrm in another binade
        inv = rn32(1 / d)
        q0 = rn32(y * inv)
        e = rn32(y - q0 * d)          # fma(-q0, d, y)
        q = rn32(q0 + e * inv)        # fma(e, inv, q0)
        if q != rn32(y / d): bad += 1
print("mismatches", bad, "of", 128*128)
