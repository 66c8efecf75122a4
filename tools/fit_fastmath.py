"""Fit the polynomial cores of csrc/fastmath.hpp (run offline; prints C++ constants).

atan(t)   = t + t*s*QA(s),            s = t^2,  |t| <= 1
sin(r)    = r + r*s*QS(s),            s = r^2,  |r| <= pi/4
cos(r)    = 1 - s/2 + s^2*QC(s),      s = r^2,  |r| <= pi/4
sin(a)    = a + a*s*QW(s),            s = a^2,  |a| <= 3   (no range reduction: tire sin)
Chebyshev fits in mpmath at 60 digits; the max error is then measured with the
coefficients rounded to double and the final assembly done in float64.
"""
import sys
import mpmath as mp
import numpy as np

mp.mp.dps = 60


def fit(f, a, b, n):
    poly, err = mp.chebyfit(f, [a, b], n, error=True)
    return [float(c) for c in poly[::-1]], err    # ascending order


def QA(s):
    if s == 0:
        return mp.mpf(-1) / 3
    t = mp.sqrt(s)
    return (mp.atan(t) / t - 1) / s


def QS(s):
    if s == 0:
        return mp.mpf(-1) / 6
    r = mp.sqrt(s)
    return (mp.sin(r) / r - 1) / s


def QC(s):
    if s == 0:
        return mp.mpf(1) / 24
    r = mp.sqrt(s)
    return (mp.cos(r) - 1 + s / 2) / s ** 2


def horner(c, x):
    acc = np.zeros_like(x) + c[-1]
    for k in reversed(c[:-1]):
        acc = acc * x + k
    return acc


def check(name, c, fn, ref, lo, hi, m=20001):
    xs = np.linspace(lo, hi, m)
    got = fn(xs, c)
    want = np.array([float(ref(mp.mpf(float(x)))) for x in xs])
    rel = np.abs(got - want) / np.maximum(np.abs(want), 1e-300)
    ulp = np.abs(got - want) / np.spacing(np.abs(want))
    print(f"  {name}: max rel {rel.max():.3e}  max ulp {ulp.max():.2f}", file=sys.stderr)


out = {}
for nA in (20, 21, 22, 23):
    cA, eA = fit(QA, 0, 1, nA)
    print(f"QA n={nA} chebyfit err {float(eA):.3e}", file=sys.stderr)
cA, _ = fit(QA, 0, 1, 22)
r4 = float(mp.pi / 4)
for nS in (7, 8, 9):
    cS, eS = fit(QS, 0, r4 * r4, nS)
    cC, eC = fit(QC, 0, r4 * r4, nS)
    print(f"QS/QC n={nS} errs {float(eS):.3e} {float(eC):.3e}", file=sys.stderr)
cS, _ = fit(QS, 0, r4 * r4, 8)
cC, _ = fit(QC, 0, r4 * r4, 8)

# reduced atan of the rollout's fast cores: |t| <= tan(pi/8) after
# atan(r) = pi/4 + atan((r - 1)/(r + 1)) for r > tan(pi/8) (fastmath.hpp atan_red)
T8 = mp.tan(mp.pi / 8)
for nR in (9, 10, 11, 12):
    cR, eR = fit(QA, 0, T8 * T8, nR)
    print(f"QR n={nR} chebyfit err {float(eR):.3e}", file=sys.stderr)
cR, _ = fit(QA, 0, T8 * T8, 10)

cW, eW = fit(QS, 0, 9.0, 10)
print(f"QW n=10 chebyfit err {float(eW):.3e}", file=sys.stderr)

atan_f = lambda t, c: t + t * (t * t) * horner(c, t * t)
sin_f = lambda r, c: r + r * (r * r) * horner(c, r * r)
cos_f = lambda r, c: 1 - (r * r) / 2 + (r * r) ** 2 * horner(c, r * r)
check("atan [0,1]", cA, atan_f, mp.atan, 1e-8, 1.0)
check("atan_red [0,tan(pi/8)]", cR, atan_f, mp.atan, 1e-8, float(T8))


def atan_red_f(r, c):
    s = r > float(T8)
    num = np.where(s, r - 1.0, r)
    den = np.where(s, r + 1.0, 1.0)
    t = num / den
    return np.where(s, float(mp.pi / 4), 0.0) + atan_f(t, c)


check("atan_red reduced [0,1]", cR, atan_red_f, mp.atan, 1e-8, 1.0)
check("sin [0,pi/4]", cS, sin_f, mp.sin, 1e-8, r4)
check("cos [0,pi/4]", cC, cos_f, mp.cos, 0.0, r4)
check("sin [0,2]", cW, sin_f, mp.sin, 1e-8, 2.0)
check("sin [0,3]", cW, sin_f, mp.sin, 1e-8, 3.0)

def emit(name, c):
    body = ",\n    ".join(f"{x!r}" for x in c)
    print(f"constexpr double {name}[{len(c)}] = {{\n    {body}}};")

emit("kAtanQ", cA)
emit("kAtanR", cR)
print(f"constexpr double kTanPi8 = {float(T8)!r};")
emit("kSinQ", cS)
emit("kCosQ", cC)
emit("kSinWQ", cW)
# Cody-Waite split of pi/2 (26+26+rest bits) for |k| <= 2^20
pio2 = mp.pi / 2
h = float(mp.mpf(int(pio2 * 2 ** 26)) / 2 ** 26)
m_ = float(mp.mpf(int((pio2 - h) * 2 ** 52)) / 2 ** 52)
l = float(pio2 - h - m_)
print(f"constexpr double kPio2Hi = {h!r}, kPio2Mid = {m_!r}, kPio2Lo = {l!r};")
print(f"constexpr double kTwoOverPi = {float(2 / mp.pi)!r}, kPio2 = {float(pio2)!r}, kPio4 = {float(mp.pi/4)!r};")
