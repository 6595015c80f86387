"""Generate the polynomial coefficients of csrc/sr_libm.h (near-minimax Chebyshev fits, mpmath).

Each fit is printed with its bound; the C++ header embeds the printed hex doubles.
  exp(r), |r| <= ln2/2          : P(r), degree 9              (|rel err| ~ 2^-46)
  sin(y) = y + y^3 S(y^2)       : S degree 4 on y^2 <= (pi/4)^2
  cos(y) = 1 - y^2/2 + y^4 C(y^2): C degree 4
  log1p(f) = f - f^2/2 + f^3 L(f), f in [sqrt(1/2) - 1, sqrt(2) - 1]: L degree 14
"""
import mpmath as mp

mp.mp.prec = 1200


def twopi_words(n=12):
    v = 2 / mp.pi
    out = []
    for _ in range(n):
        v *= 2 ** 32
        w = int(mp.floor(v))
        out.append(w)
        v -= w
    return out


def fit(f, a, b, deg):
    with mp.workprec(300):
        poly, err = mp.chebyfit(f, [a, b], deg + 1, error=True)
    return [float(c) for c in poly], float(err)  # highest degree first


def main():
    print("2/pi words:", ", ".join("0x%08Xu" % w for w in twopi_words()))
    h = mp.log(2) / 2
    zmax = (mp.pi / 4) ** 2
    fits = {
        "EXP": fit(mp.exp, -h, h, 9),
        "SIN": fit(lambda z: (mp.sin(mp.sqrt(z)) - mp.sqrt(z)) / (z * mp.sqrt(z)) if z > 0 else mp.mpf(-1) / 6, 0, zmax, 4),
        "COS": fit(lambda z: (mp.cos(mp.sqrt(z)) - 1 + z / 2) / (z * z) if z > 0 else mp.mpf(1) / 24, 0, zmax, 4),
        "LOG": fit(lambda f: (mp.log1p(f) - f + f * f / 2) / f ** 3 if f != 0 else mp.mpf(1) / 3,
                   mp.sqrt(mp.mpf(1) / 2) - 1, mp.sqrt(2) - 1, 14),
    }
    for name, (c, err) in fits.items():
        print(f"// {name}: degree {len(c) - 1}, fit error {err:.3e}")
        print(f"constexpr double k{name}[{len(c)}] = {{" + ", ".join(float.hex(v) for v in c) + "};")
    print("pi/2 split:", [float.hex(float(x)) for x in split(mp.pi / 2, 3)])
    print("ln2 split:", [float.hex(float(x)) for x in split(mp.log(2), 2)])
    print("log2(e):", float.hex(float(1 / mp.log(2))), " 2/pi:", float.hex(float(2 / mp.pi)))


def split(v, k):
    out = []
    for _ in range(k):
        d = mp.mpf(float(v))
        out.append(d)
        v -= d
    return out


if __name__ == "__main__":
    main()


def tables():
    """Tables of csrc/sr_libm.h: sin/cos(k pi/64), k = 0..127; log: for the 32 mantissa cells of
    [1, 2), invc = 1 / (cell centre) rounded to double and logc = -log(invc) (so that
    log(m) = logc + log1p(m * invc - 1) holds exactly in real arithmetic); cells of [1.5, 2) serve
    m/2 (centre halved), cell 0 has centre 1."""
    trig = [(float(mp.sin(k * mp.pi / 64)), float(mp.cos(k * mp.pi / 64))) for k in range(128)]
    logt = []
    for k in range(32):
        c = 1 + (mp.mpf(k) + mp.mpf(1) / 2) / 32
        if k == 0:  # cell [1, 1 + 1/32): centre 1 exactly, so log(1) = 0 exactly
            c = mp.mpf(1)
        elif k >= 16:  # m in [1.5, 2) is taken as m/2 in [0.75, 1) with e + 1 (no cancellation near 1-)
            c = c / 2
        invc = float(1 / c)
        logt.append((invc, float(-mp.log(mp.mpf(invc)))))
    return trig, logt


def emit_tables():
    trig, logt = tables()
    print("constexpr double kTrigTab[256] = {" + ", ".join(float.hex(v) for p in trig for v in p) + "};")
    print("constexpr double kLogTab[64] = {" + ", ".join(float.hex(v) for p in logt for v in p) + "};")
    h = mp.pi / 1024  # reduction by 16 n' (pi / 1024) = n' pi / 64: the shifter's low word is 16 n'
    print("pi/1024 split:", [float.hex(float(x)) for x in split(h, 3)], " 1024/pi:", float.hex(float(1024 / mp.pi)))
    # polynomial bounds on |r| <= pi/128 (trig, Taylor to r^5 / r^4) and |r| <= 1/32 (log, to r^7)
    r = mp.pi / 128
    print("trig s rel err:", float(r ** 6 / mp.factorial(7)), " c err:", float(r ** 6 / mp.factorial(6)))
    r = mp.mpf(1) / 32
    print("log rel err (deg 7):", float(r ** 7 / 8))


if __name__ == "__main__" and len(__import__("sys").argv) > 1:
    emit_tables()
