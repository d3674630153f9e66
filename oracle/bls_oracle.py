"""CPU restatement of the BLS12-381 pairing behind threshold-decrypt share
verification.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker -- never by the product path
(hbbft_amd/).  Pure Python integers, written for clarity, not speed
(a pairing takes ~0.1-0.3 s here).

What it restates, and from where
--------------------------------
hbbft calls (`/root/reference/src/threshold_decrypt.rs:142, 220-228`):

    Ciphertext::verify(ct)                  e(G1::one(), W)  == e(U, hash_g1_g2(U, V))
    PublicKeyShare::verify_decryption_share e(share, hash)   == e(pk_i, W)

from `threshold_crypto` (git rev 624eeee, `/root/reference/Cargo.toml:36`),
whose `PEngine::pairing` is the `pairing` crate's BLS12-381 (zkcrypto
`pairing` 0.14/0.15 series) -- neither crate is vendored in /root/reference,
so this is a restatement of their published algorithm:

* curve      E : y^2 = x^3 + 4 over Fp;  twist E' : y^2 = x^3 + 4(u+1) over
               Fp2 = Fp[u]/(u^2+1) (an M-type sextic twist)
* pairing    optimal ate, Miller loop over |x|, x = -0xd201000000010000,
               conjugated because x < 0 (pairing `Bls12::miller_loop`)
* final exp  the easy part f^((p^6-1)(p^2+1)) followed by the crate's
               hard-part chain (`Bls12::final_exponentiation`, restated in
               `final_exponentiation` below); the chain evaluates
               f^(3 (p^4-p^2+1)/r), so the crate's GT value is the standard
               reduced pairing cubed.  `tests/test_bls_oracle.py` checks this
               identity against a plain square-and-multiply of 3 (p^12-1)/r.

Any Miller-loop line scaling by a proper-subfield element is removed by the
final exponentiation, so the GT values here are independent of the Miller
formulas; the oracle uses the plainest ones (affine, in Fp12) and the HIP
kernels use projective formulas on the twist.

Parity anchors (no reference byte vector exists in /root/reference): the
standard generator coordinates (on-curve and r-torsion checked here),
bilinearity, non-degeneracy, e^r = 1, and the chain identity above.  The
GT *bytes* of the crate are therefore "parity unpinned"; the boolean
outcomes hbbft consumes are pinned by bilinearity.

Representation: Fp12 is Fp[w]/(w^12 - 2 w^6 + 2) (w^6 = u + 1 = xi, u^2 = -1),
a list of 12 coefficients of 1, w, ..., w^11.  `to_tower` converts to the
crate's tower Fp12 = Fp6[w]/(w^2 - v), Fp6 = Fp2[v]/(v^3 - xi):
c0 = (w^0, w^2, w^4), c1 = (w^1, w^3, w^5) as Fp2 coefficients.
"""

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
X_ABS = 0xd201000000010000          # |x|; x is negative for BLS12-381
X_NEG = True

G1_GEN = (
    0x17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb,
    0x08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1,
)
G2_GEN = (
    (0x024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8,
     0x13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e),
    (0x0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801,
     0x0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be),
)


def inv(a):
    return pow(a, P - 2, P)


# ---------------------------------------------------------------- Fp2 = Fp[u]/(u^2+1)
def f2add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2inv(a):
    t = inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2eq(a, b):
    return a[0] % P == b[0] % P and a[1] % P == b[1] % P


F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (1, 1)                 # u + 1
B1 = 4
B2 = (4, 4)                 # 4 (u + 1)


# ---------------------------------------------------------------- G1 / G2 (affine, None = infinity)
def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return f2eq(f2mul(y, y), f2add(f2mul(f2mul(x, x), x), B2))


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * inv(2 * a[1]) % P
    else:
        lam = (b[1] - a[1]) * inv(b[0] - a[0]) % P
    x = (lam * lam - a[0] - b[0]) % P
    return (x, (lam * (a[0] - x) - a[1]) % P)


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if f2eq(a[0], b[0]):
        if f2eq(f2add(a[1], b[1]), F2_ZERO):
            return None
        x2 = f2mul(a[0], a[0])
        lam = f2mul((3 * x2[0] % P, 3 * x2[1] % P), f2inv(f2add(a[1], a[1])))
    else:
        lam = f2mul(f2sub(b[1], a[1]), f2inv(f2sub(b[0], a[0])))
    x = f2sub(f2sub(f2mul(lam, lam), a[0]), b[0])
    return (x, f2sub(f2mul(lam, f2sub(a[0], x)), a[1]))


def _smul(add, pt, k):
    acc = None
    while k:
        if k & 1:
            acc = add(acc, pt)
        pt = add(pt, pt)
        k >>= 1
    return acc


def g1_mul(pt, k):
    return _smul(g1_add, pt, k % R)


def g2_mul(pt, k):
    return _smul(g2_add, pt, k % R)


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


# ---------------------------------------------------------------- subgroup membership
# The crate's deserialisation (`EncodedPoint::into_affine`) checks the curve
# equation and then `is_in_correct_subgroup_assuming_on_curve`: [r] P == O
# (the order-r subgroup; E(Fp) has cofactor h1, E'(Fp2) cofactor h2).  The HIP
# decoders use the equivalent endomorphism tests (pairing.hip); the tests
# compare both on points inside and outside the subgroup.
def g1_in_subgroup(pt):
    return pt is None or (g1_on_curve(pt) and _smul(g1_add, pt, R) is None)


def g2_in_subgroup(pt):
    return pt is None or (g2_on_curve(pt) and _smul(g2_add, pt, R) is None)


BETA = 0x5f19672fdf76ce51ba69c6076a0f77eaddb3a93be6f89688de17d813620a00022e01fffffffefffe


def g1_endo_test(pt):
    """Scott's G1 test: phi(P) = (beta x, y) == -[x^2] P."""
    return (BETA * pt[0] % P, pt[1]) == g1_neg(_smul(g1_add, pt, X_ABS * X_ABS))


def _f2pow(a, e):
    out = F2_ONE
    while e:
        if e & 1:
            out = f2mul(out, a)
        a = f2mul(a, a)
        e >>= 1
    return out


def psi(q):
    """Untwist-Frobenius-twist on E': (conj(x) xi^-((p-1)/3), conj(y) xi^-((p-1)/2))."""
    cx, cy = f2inv(_f2pow(XI, (P - 1) // 3)), f2inv(_f2pow(XI, (P - 1) // 2))
    x, y = q
    return (f2mul((x[0], (-x[1]) % P), cx), f2mul((y[0], (-y[1]) % P), cy))


def g2_endo_test(q):
    """Scott's G2 test: psi(Q) == [x] Q = -[|x|] Q."""
    t = _smul(g2_add, q, X_ABS)
    return t is not None and psi(q) == (t[0], f2neg(t[1]))


def _f2sqrt(a):
    """Square root in Fp2 (p = 3 mod 4), or None."""
    a1 = _f2pow(a, (P - 3) // 4)
    alpha = f2mul(f2mul(a1, a1), a)
    x0 = f2mul(a1, a)
    if f2eq(alpha, (P - 1, 0)):
        x = f2mul((0, 1), x0)
    else:
        x = f2mul(_f2pow(f2add(F2_ONE, alpha), (P - 1) // 2), x0)
    return x if f2eq(f2mul(x, x), a) else None


def g1_curve_point(seed):
    """A point of E(Fp) from a seed (the first x >= seed on the curve), almost
    surely outside G1 (the probability of landing in it is 1/h1)."""
    x = seed % P
    while True:
        a = (x * x * x + B1) % P
        y = pow(a, (P + 1) // 4, P)
        if y * y % P == a:
            return (x, y)
        x += 1


def g2_curve_point(seed):
    """A point of E'(Fp2) from a seed, almost surely outside G2."""
    x = (seed % P, 1)
    while True:
        y = _f2sqrt(f2add(f2mul(f2mul(x, x), x), B2))
        if y is not None:
            return (x, y)
        x = (x[0] + 1, 1)


# ---------------------------------------------------------------- Fp12 = Fp[w]/(w^12 - 2w^6 + 2)
def f12(coeffs):
    return [c % P for c in coeffs]


F12_ONE = [1] + [0] * 11


def f12mul(a, b):
    t = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                t[i + j] += ai * bj
    for k in range(22, 11, -1):     # w^k = 2 w^(k-6) - 2 w^(k-12)
        c = t[k]
        if c:
            t[k - 6] += 2 * c
            t[k - 12] -= 2 * c
    return [c % P for c in t[:12]]


def f12sub(a, b):
    return [(x - y) % P for x, y in zip(a, b)]


def _poly_trim(a):
    while a and a[-1] % P == 0:
        a.pop()
    return a


def _poly_divmod(a, b):
    a = [x % P for x in a]
    q = [0] * max(len(a) - len(b) + 1, 1)
    ib = inv(b[-1])
    while len(_poly_trim(a)) >= len(b):
        d = len(a) - len(b)
        c = a[-1] * ib % P
        q[d] = c
        for i, bi in enumerate(b):
            a[i + d] = (a[i + d] - c * bi) % P
    return q, a


def f12inv(a):
    """Extended Euclid in Fp[w] against the modulus w^12 - 2w^6 + 2."""
    mod = [2, 0, 0, 0, 0, 0, P - 2, 0, 0, 0, 0, 0, 1]
    r0, r1 = mod[:], _poly_trim([x % P for x in a])
    s0, s1 = [0], [1]
    assert r1, "inverse of zero"
    while len(r1) > 1:
        q, rem = _poly_divmod(r0, r1)
        qs = [0] * (len(q) + len(s1))
        for i, qi in enumerate(q):
            for j, sj in enumerate(s1):
                qs[i + j] += qi * sj
        s2 = [((s0[i] if i < len(s0) else 0) - (qs[i] if i < len(qs) else 0)) % P
              for i in range(max(len(s0), len(qs)))]
        r0, r1, s0, s1 = r1, _poly_trim(rem), s1, _poly_trim(s2)
    c = inv(r1[0])
    out = [x * c % P for x in s1] + [0] * 12
    return _reduce12(out)


def _reduce12(t):
    t = list(t) + [0] * max(0, 23 - len(t))
    for k in range(len(t) - 1, 11, -1):
        c = t[k]
        if c:
            t[k - 6] += 2 * c
            t[k - 12] -= 2 * c
        t[k] = 0
    return [c % P for c in t[:12]]


def f12pow(a, e):
    out = F12_ONE
    for bit in bin(e)[2:]:
        out = f12mul(out, out)
        if bit == "1":
            out = f12mul(out, a)
    return out


def f12conj(a):
    """a^(p^6): w^(p^6) = -w (w^6 = xi and xi^((p^6-1)/6) = -1), so odd powers flip."""
    return [c if i % 2 == 0 else (-c) % P for i, c in enumerate(a)]


# w^(i p^k) as Fp12 elements, for the Frobenius map
def _frob_table(k):
    pk = P ** k
    # w^(p^k) = w * (w^6)^((p^k-1)/6) = w * xi^((p^k-1)/6); xi is in Fp2 (coeffs 1, w^6)
    g = _f2pow(XI, (pk - 1) // 6)
    wp = [0] * 12
    wp[1] = g[0]            # g0 * w
    wp[7] = g[1]            # g1 * u * w, u = w^6 - 1  ->  g1 (w^7 - w)
    wp[1] = (wp[1] - g[1]) % P
    out = [F12_ONE]
    for _ in range(11):
        out.append(f12mul(out[-1], wp))
    return out


def _f2pow(a, e):
    out = F2_ONE
    while e:
        if e & 1:
            out = f2mul(out, a)
        a = f2mul(a, a)
        e >>= 1
    return out


_FROB = {}


def f12frob(a, k):
    """a^(p^k): the coefficients are in Fp, so only the basis moves."""
    if k not in _FROB:
        _FROB[k] = _frob_table(k)
    tab = _FROB[k]
    out = [0] * 12
    for i, c in enumerate(a):
        if c:
            for j, t in enumerate(tab[i]):
                out[j] += c * t
    return [c % P for c in out]


# ---------------------------------------------------------------- embedding and lines
def _fp2_to_f12(a):
    """a0 + a1 u with u = w^6 - 1."""
    t = [0] * 12
    t[0] = (a[0] - a[1]) % P
    t[6] = a[1] % P
    return t


_W_INV = None


def _untwist(q):
    """psi: E'(Fp2) -> E(Fp12), (x, y) -> (x / w^2, y / w^3)."""
    global _W_INV
    if _W_INV is None:
        w = [0] * 12
        w[1] = 1
        _W_INV = f12inv(w)
    wi2 = f12mul(_W_INV, _W_INV)
    wi3 = f12mul(wi2, _W_INV)
    return (f12mul(_fp2_to_f12(q[0]), wi2), f12mul(_fp2_to_f12(q[1]), wi3))


def _const12(c):
    return [c % P] + [0] * 11


def miller_loop(p1, q2):
    """f_{|x|, psi(Q)}(P) with affine Fp12 lines, conjugated for x < 0
    (pairing crate `Bls12::miller_loop`).  Infinity on either side gives 1."""
    if p1 is None or q2 is None:
        return F12_ONE
    xp, yp = _const12(p1[0]), _const12(p1[1])
    Q = _untwist(q2)
    T = Q
    f = F12_ONE
    three = _const12(3)
    for bit in bin(X_ABS)[3:]:
        # tangent at T
        lam = f12mul(f12mul(three, f12mul(T[0], T[0])), f12inv(f12mul(_const12(2), T[1])))
        line = f12sub(f12sub(yp, T[1]), f12mul(lam, f12sub(xp, T[0])))
        f = f12mul(f12mul(f, f), line)
        x3 = f12sub(f12sub(f12mul(lam, lam), T[0]), T[0])
        T = (x3, f12sub(f12mul(lam, f12sub(T[0], x3)), T[1]))
        if bit == "1":
            lam = f12mul(f12sub(Q[1], T[1]), f12inv(f12sub(Q[0], T[0])))
            line = f12sub(f12sub(yp, T[1]), f12mul(lam, f12sub(xp, T[0])))
            f = f12mul(f, line)
            x3 = f12sub(f12sub(f12mul(lam, lam), T[0]), Q[0])
            T = (x3, f12sub(f12mul(lam, f12sub(T[0], x3)), T[1]))
    return f12conj(f) if X_NEG else f


def _exp_by_x(f, e):
    out = f12pow(f, e)
    return f12conj(out) if X_NEG else out


def final_exponentiation(f):
    """The pairing crate's `Bls12::final_exponentiation`: easy part, then its
    hard-part chain (restated step by step; = f^(3 (p^12-1)/r))."""
    f1 = f12conj(f)
    f2 = f12inv(f)
    r = f12mul(f1, f2)              # f^(p^6 - 1)
    f2 = r
    r = f12frob(r, 2)
    r = f12mul(r, f2)               # ^(p^2 + 1)
    x = X_ABS
    y0 = f12mul(r, r)
    y1 = _exp_by_x(y0, x)
    y2 = _exp_by_x(y1, x >> 1)
    y3 = f12conj(r)
    y1 = f12mul(y1, y3)
    y1 = f12conj(y1)
    y1 = f12mul(y1, y2)
    y2 = _exp_by_x(y1, x)
    y3 = _exp_by_x(y2, x)
    y1 = f12conj(y1)
    y3 = f12mul(y3, y1)
    y1 = f12conj(y1)
    y1 = f12frob(y1, 3)
    y2 = f12frob(y2, 2)
    y1 = f12mul(y1, y2)
    y2 = _exp_by_x(y3, x)
    y2 = f12mul(y2, y0)
    y2 = f12mul(y2, r)
    y1 = f12mul(y1, y2)
    y2 = f12frob(y3, 1)
    y1 = f12mul(y1, y2)
    return y1


def final_exponentiation_plain(f, power=3):
    """f^(power (p^12-1)/r) by square-and-multiply (the chain's specification)."""
    easy = f12mul(f12conj(f), f12inv(f))
    easy = f12mul(f12frob(easy, 2), easy)
    return f12pow(easy, power * (P ** 4 - P ** 2 + 1) // R)


def pairing(p1, q2):
    return final_exponentiation(miller_loop(p1, q2))


def pairing_check(a, b, c, d):
    """e(a, b) == e(c, d), as `verify_decryption_share` / `Ciphertext::verify`
    evaluate it (two pairings compared in GT)."""
    return pairing(a, b) == pairing(c, d)


# ---------------------------------------------------------------- tower layout and encodings
def to_tower(a):
    """[(c0.c0), (c0.c1), (c0.c2), (c1.c0), (c1.c1), (c1.c2)] as Fp2 pairs: the
    crate's Fp12 = Fp6[w]/(w^2 - v), Fp6 = Fp2[v]/(v^3 - xi) coefficient order."""
    out = []
    for e in (0, 2, 4, 1, 3, 5):
        # coefficient of w^e over Fp2: a_e + a_{e+6} w^6 = (a_e + a_{e+6}) + a_{e+6} u
        out.append(((a[e] + a[e + 6]) % P, a[e + 6] % P))
    return out


def from_tower(t):
    a = [0] * 12
    for e, c in zip((0, 2, 4, 1, 3, 5), t):
        a[e] = (c[0] - c[1]) % P
        a[e + 6] = c[1] % P
    return a


def fp_bytes(v):
    return (v % P).to_bytes(48, "big")


def gt_bytes(a):
    """576 bytes: the 12 Fp coefficients of the tower form, each big-endian,
    in the order c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1."""
    return b"".join(fp_bytes(c[0]) + fp_bytes(c[1]) for c in to_tower(a))


def g1_bytes(pt):
    """Uncompressed G1 encoding (zkcrypto `G1Uncompressed`): x || y big-endian,
    96 bytes; the point at infinity sets flag bit 0x40 of byte 0, rest zero."""
    if pt is None:
        return b"\x40" + b"\0" * 95
    return fp_bytes(pt[0]) + fp_bytes(pt[1])


def g2_bytes(pt):
    """Uncompressed G2 encoding (zkcrypto `G2Uncompressed`): x.c1 || x.c0 ||
    y.c1 || y.c0 big-endian, 192 bytes; infinity = flag 0x40 in byte 0."""
    if pt is None:
        return b"\x40" + b"\0" * 191
    (x0, x1), (y0, y1) = pt
    return fp_bytes(x1) + fp_bytes(x0) + fp_bytes(y1) + fp_bytes(y0)


# ---------------------------------------------------------------- threshold decryption shapes
def decryption_share_case(sk, r_enc, h_scalar, tamper=False):
    """A (share, pk_share, hash, W) tuple with the shapes of
    `verify_decryption_share` (threshold_crypto): U = r G1, W = r H, share = sk U,
    pk = sk G1; H = h G2 stands for hash_g1_g2(U, V) (a G2 point the host
    computes).  `tamper` offsets the share by G1, so the check fails."""
    H = g2_mul(G2_GEN, h_scalar)
    U = g1_mul(G1_GEN, r_enc)
    W = g2_mul(H, r_enc)
    share = g1_mul(U, sk)
    if tamper:
        share = g1_add(share, G1_GEN)
    pk = g1_mul(G1_GEN, sk)
    return share, H, pk, W
