"""Generates the 87 cached powers of ten (10^(-348 + 8i), 64-bit significand rounded to nearest,
binary exponent) that the Grisu2 restatement in pixie_amd/host/json_double.h uses.  Exact
rational arithmetic; the printed table is pasted into the header."""
from fractions import Fraction
import math


def cached(k):
    v = Fraction(10) ** k
    e = math.floor(math.log2(v.numerator) - math.log2(v.denominator)) - 63
    while v / Fraction(2) ** e >= 2 ** 64:
        e += 1
    while v / Fraction(2) ** e < 2 ** 63:
        e -= 1
    q = v / Fraction(2) ** e
    f = q.numerator // q.denominator
    if q - f >= Fraction(1, 2):
        f += 1
    return f, e


if __name__ == "__main__":
    rows = [cached(-348 + 8 * i) for i in range(87)]
    print("static const uint64_t kPow10F[87] = {")
    for i in range(0, 87, 3):
        print("    " + ", ".join("0x%016xULL" % f for f, _ in rows[i:i + 3]) + ",")
    print("};")
    print("static const int16_t kPow10E[87] = {")
    for i in range(0, 87, 12):
        print("    " + ", ".join(str(e) for _, e in rows[i:i + 12]) + ",")
    print("};")
