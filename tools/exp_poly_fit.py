"""Minimax (relative error) degree-2 polynomial for 2^(f/4096) on f in [0, 1]:
the coefficients of exp2_4096_poly01 in svgd_kernels.hip (the biased-exponent
row stream, whose range reduction yields f = fract(u) in [0, 1)).  Remez
exchange in long double; prints the coefficients and their hex forms."""
import numpy as np
L = np.longdouble
a = np.log(L(2)) / L(4096)
def target(f): return np.exp(a * f)
# minimax relative error, degree 2 on [0,1]
xs = np.array([0, 0.15, 0.5, 0.85, 1.0], dtype=L)  # 4 points for deg2 + E (n+2=4)
xs = np.array([0, 0.25, 0.75, 1.0], dtype=L)
for it in range(30):
    A = np.zeros((4, 4), dtype=L)
    b = np.zeros(4, dtype=L)
    for i, x in enumerate(xs):
        t = target(x)
        A[i, :3] = [1, x, x * x]
        A[i, 3] = (-1) ** i * t
        b[i] = t
    sol = np.linalg.solve(A.astype(np.float64), b.astype(np.float64))  # solve in double first
    # refine in longdouble via simple iteration
    c = sol[:3].astype(L)
    g = np.linspace(0, 1, 20001, dtype=L)
    err = (c[0] + c[1] * g + c[2] * g * g) / target(g) - 1
    # new extrema
    idx = [0]
    for i in range(1, len(g) - 1):
        if (err[i] - err[i - 1]) * (err[i + 1] - err[i]) < 0: idx.append(i)
    idx.append(len(g) - 1)
    if len(idx) == 4: xs = g[idx]
print("coeffs", [float(x) for x in c], "max rel err", float(np.max(np.abs(err))))
cd = [float(x) for x in c]
print([x.hex() for x in cd])
