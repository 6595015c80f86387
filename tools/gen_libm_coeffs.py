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
    """Tables of csrc/sr_libm.h: sin/cos(k pi/64), k = 0..127; log: 64 cells of the offset octave
    z in [0x3f330000, 0x3fb30000) (Float32 bits; x = 2^k z with z ~ [0.699, 1.398), so no branch
    between the halves of the octave), cell i = bits [OFF + i 2^17, OFF + (i+1) 2^17):
    invc = 1 / (cell centre) rounded to double and logc = -log(invc) (so that
    log(z) = logc + log1p(z * invc - 1) holds exactly in real arithmetic); the cell holding 1
    (i = 38) has centre 1, so log(1) = 0 exactly.  |z invc - 1| <= 2^-7 in every cell."""
    import struct

    def f32(bits):
        return mp.mpf(struct.unpack("<f", struct.pack("<I", bits))[0])

    trig = [(float(mp.sin(k * mp.pi / 64)), float(mp.cos(k * mp.pi / 64))) for k in range(128)]
    logt, rmax = [], mp.mpf(0)
    for i in range(64):
        lo, hi = f32(LOG_OFF + (i << 17)), f32(LOG_OFF + ((i + 1) << 17))
        c = mp.mpf(1) if lo <= 1 < hi else (lo + hi) / 2
        invc = float(1 / c)
        rmax = max(rmax, abs(lo * invc - 1), abs(hi * invc - 1))
        logt.append((invc, float(-mp.log(mp.mpf(invc)))))
    return trig, logt, rmax


LOG_OFF = 0x3F330000


def emit_tables():
    trig, logt, rmax = tables()
    print("constexpr double kTrigTab[256] = {" + ", ".join(float.hex(v) for p in trig for v in p) + "};")
    print("constexpr double kLogTab[128] = {" + ", ".join(float.hex(v) for p in logt for v in p) + "};")
    h = mp.pi / 1024  # reduction by 16 n' (pi / 1024) = n' pi / 64: the shifter's low word is 16 n'
    print("pi/1024 split:", [float.hex(float(x)) for x in split(h, 3)], " 1024/pi:", float.hex(float(1024 / mp.pi)))
    # polynomial bounds on |r| <= pi/128 (trig, Taylor to r^5 / r^4) and |r| <= 1/32 (log, to r^7)
    r = mp.pi / 128
    print("trig s rel err:", float(r ** 6 / mp.factorial(7)), " c err:", float(r ** 6 / mp.factorial(6)))
    # log1p(r) by Taylor to r^6: |error| <= |r|^7 / 7 absolute, relative to |log x| >= |log(0.99609375)|
    # outside the centre-1 cell and to |r| inside it
    print("log |r| max:", float(rmax), " abs err:", float(rmax ** 7 / 7),
          " rel err (worst cell):", float(rmax ** 7 / 7 / abs(mp.log(mp.mpf(0.99609375)))))


if __name__ == "__main__" and len(__import__("sys").argv) > 1:
    emit_tables()
