"""Print the double-double constants of csrc/htp_libm.h (pi splits, 1/n!, 1/(2n+1), atan(i/16), log(1+i/32),
ln 2 splits), computed with mpmath at 300 bits.  python tools/gen_libm_consts.py > /tmp/c.txt"""
import mpmath

mpmath.mp.prec = 300


def dd(v):
    hi = float(v)
    lo = float(v - mpmath.mpf(hi))
    return hi, lo


def split3(v):
    a = float(v)
    b = float(v - a)
    c = float(v - a - b)
    return a, b, c


def f(x):
    return repr(float(x)) if float(x) != 0 else "0.0"


def emit_dd(name, vals):
    print(f"constexpr double {name}[{len(vals)}][2] = {{")
    for v in vals:
        h, l = dd(v)
        print(f"    {{{f(h)}, {f(l)}}},")
    print("};")


pi = mpmath.pi
print("// pi/2 = PIO2_1 + PIO2_2 + PIO2_3 (+ 2^-160)")
a, b, c = split3(pi / 2)
print(f"constexpr double PIO2_1 = {f(a)}, PIO2_2 = {f(b)}, PIO2_3 = {f(c)};")
h, l = dd(pi)
print(f"constexpr double PI_H = {f(h)}, PI_L = {f(l)};")
h, l = dd(pi / 2)
print(f"constexpr double PIO2_H = {f(h)}, PIO2_L = {f(l)};")
h, l = dd(pi / 4)
print(f"constexpr double PIO4_H = {f(h)}, PIO4_L = {f(l)};")
h, l = dd(3 * pi / 4)
print(f"constexpr double PI34_H = {f(h)}, PI34_L = {f(l)};")
print(f"constexpr double TWO_OVER_PI = {f(2 / pi)};")
a, b, c = split3(mpmath.log(2))
print(f"constexpr double LN2_1 = {f(a)}, LN2_2 = {f(b)}, LN2_3 = {f(c)};")
print(f"constexpr double INV_LN2 = {f(1 / mpmath.log(2))};")
emit_dd("SIN_C", [(-1) ** n / mpmath.factorial(2 * n + 1) for n in range(14)])
emit_dd("COS_C", [(-1) ** n / mpmath.factorial(2 * n) for n in range(15)])
emit_dd("ATAN_C", [(-1) ** n / mpmath.mpf(2 * n + 1) for n in range(12)])
emit_dd("ATANH_C", [1 / mpmath.mpf(2 * n + 1) for n in range(12)])
emit_dd("EXP_C", [1 / mpmath.factorial(n) for n in range(14)])
emit_dd("ATAN_T", [mpmath.atan(mpmath.mpf(i) / 16) for i in range(17)])
emit_dd("LOG_T", [mpmath.log(1 + mpmath.mpf(i) / 32) for i in range(-8, 17)])
