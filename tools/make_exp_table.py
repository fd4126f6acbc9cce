"""Generate the exp2 table and polynomial coefficients used by exp2_256()
in svgdcpp_amd/csrc/svgd_kernels.hip (printed as C hex-float literals).

T[i] = 2^(i/256), i = 0..255, correctly rounded to double (Decimal at 60
digits, then Python's correctly rounded Decimal -> float conversion).
c_m = (ln 2 / 256)^m / m!, m = 0..5 (the Taylor coefficients of 2^(f/256)).
"""
from decimal import Decimal, getcontext


def table():
    getcontext().prec = 60
    ln2 = Decimal(2).ln()
    return [float((Decimal(i) / 256 * ln2).exp()) for i in range(256)]


def coeffs(m_max=5):
    getcontext().prec = 60
    x = Decimal(2).ln() / 256
    out, fact = [], 1
    for m in range(m_max + 1):
        if m:
            fact *= m
        out.append(float(x ** m / fact))
    return out


if __name__ == "__main__":
    t = table()
    print("__constant__ double EXP2_TAB256[256] = {")
    for i in range(0, 256, 4):
        print("    " + ", ".join(v.hex() for v in t[i:i + 4]) + ",")
    print("};")
    print("// coefficients:", ", ".join(c.hex() for c in coeffs()))
