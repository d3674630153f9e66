"""Threshold-decrypt share verification on the MI355X.

hbbft's `ThresholdDecrypt` (/root/reference/src/threshold_decrypt.rs) checks
every ciphertext once (`ct.verify()`, line 142) and every received decryption
share (`pk.verify_decryption_share(share, ct)`, lines 220-228), both from
`threshold_crypto` (rev 624eeee):

    Ciphertext::verify                      e(G1::one(), W) == e(U, H)
    PublicKeyShare::verify_decryption_share e(share, H)     == e(pk_i, W)

with H = hash_g1_g2(U, V), a G2 point the caller computes once per
ciphertext (SHA3-256 and a ChaCha-seeded G2 sample -- host work, not on the
bulk path).  In an epoch every node verifies N shares of each of N
ciphertexts, so the pairing checks come in batches of N^2 per node; this
module runs them through `hbrbc_pairing_check_batch` (hbbft_amd/csrc/
pairing.hip): one Miller loop per lane, one final exponentiation per check.

Points are the crate's uncompressed encodings (G1: 96 bytes, G2: 192 bytes,
big-endian; see include/hbrbc.h).  There is no CPU fallback: without the
library or a GPU the calls raise `HbrbcUnavailable`.
"""
import ctypes

from . import HbrbcUnavailable, RseError, _check, lib  # noqa: F401

G1_BYTES = 96
G2_BYTES = 192
GT_BYTES = 576

# G1::one() (the standard generator), uncompressed: the `a` of Ciphertext::verify.
G1_ONE = bytes.fromhex(
    "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"
    "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1")

CHECK_OK, CHECK_FAIL, CHECK_INVALID = 1, 0, 2


def _torch():
    import torch
    return torch


def workspace(pairings, device=0):
    """Device workspace for `pairings` Miller loops (reusable across calls)."""
    torch = _torch()
    n = lib().hbrbc_pairing_workspace_size(pairings)
    return torch.empty(max(n, 1), dtype=torch.uint8, device="cuda:%d" % device)


def _stream(dev, stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    return ctypes.c_void_p(s.cuda_stream)


def pairing_batch(g1, g2, ws=None, stream=None):
    """`PEngine::pairing(g1[i], g2[i])` for every row: g1 uint8 [n, 96], g2 uint8
    [n, 192] on one device.  Returns (gt uint8 [n, 576], status uint8 [n];
    0 ok, 2 invalid point)."""
    torch = _torch()
    n = g1.shape[0]
    assert g1.shape == (n, G1_BYTES) and g2.shape == (n, G2_BYTES), (g1.shape, g2.shape)
    assert g1.is_contiguous() and g2.is_contiguous() and g1.device == g2.device
    gt = torch.empty((n, GT_BYTES), dtype=torch.uint8, device=g1.device)
    st = torch.empty((n,), dtype=torch.uint8, device=g1.device)
    if ws is None:
        ws = workspace(n, g1.device.index)
    assert ws.numel() >= lib().hbrbc_pairing_workspace_size(n)
    _check(lib().hbrbc_pairing_batch(g1.data_ptr(), g2.data_ptr(), n, gt.data_ptr(),
                                     st.data_ptr(), ws.data_ptr(), _stream(g1.device, stream)))
    return gt, st


def pairing_check_batch(g1, g2, ws=None, stream=None):
    """count checks e(a_i, b_i) == e(c_i, d_i): g1 uint8 [2 count, 96] = a_0,
    c_0, a_1, c_1, ...; g2 uint8 [2 count, 192] = b_0, d_0, ....  Returns
    uint8 [count]: 1 equal, 0 not, 2 invalid point."""
    torch = _torch()
    n2 = g1.shape[0]
    assert n2 % 2 == 0 and g1.shape == (n2, G1_BYTES) and g2.shape == (n2, G2_BYTES)
    assert g1.is_contiguous() and g2.is_contiguous() and g1.device == g2.device
    ok = torch.empty((n2 // 2,), dtype=torch.uint8, device=g1.device)
    if ws is None:
        ws = workspace(n2, g1.device.index)
    assert ws.numel() >= lib().hbrbc_pairing_workspace_size(n2)
    _check(lib().hbrbc_pairing_check_batch(g1.data_ptr(), g2.data_ptr(), n2 // 2, ok.data_ptr(),
                                           ws.data_ptr(), _stream(g1.device, stream)))
    return ok


def g2_prepare(g2, stream=None):
    """Prepare G2 points (uint8 [n, 192]) once: the Miller-loop lines every
    check against them reuses (the crate's G2Prepared).  Returns the device
    table (uint8) for pairing_check_prepared."""
    torch = _torch()
    n = g2.shape[0]
    assert g2.shape == (n, G2_BYTES) and g2.is_contiguous()
    prep = torch.empty(max(1, lib().hbrbc_g2_prepared_size(n)), dtype=torch.uint8,
                       device=g2.device)
    _check(lib().hbrbc_g2_prepare(g2.data_ptr(), n, prep.data_ptr(), _stream(g2.device, stream)))
    return prep


def pairing_check_prepared(g1, prep, points, idx_b, idx_d, ws=None, stream=None):
    """count checks e(a_i, P[idx_b[i]]) == e(c_i, P[idx_d[i]]) against `points`
    prepared G2 points: g1 uint8 [2 count, 96] = a_0, c_0, ...; idx_* int32
    [count].  Returns uint8 [count]: 1 equal, 0 not, 2 invalid point."""
    torch = _torch()
    n2 = g1.shape[0]
    count = n2 // 2
    assert n2 % 2 == 0 and g1.shape == (n2, G1_BYTES) and g1.is_contiguous()
    assert idx_b.shape == (count,) and idx_d.shape == (count,)
    assert idx_b.dtype == torch.int32 and idx_d.dtype == torch.int32
    assert idx_b.is_contiguous() and idx_d.is_contiguous()
    # an index outside [0, points) makes that check's outcome 2 (invalid) on the device
    ok = torch.empty((count,), dtype=torch.uint8, device=g1.device)
    if ws is None:
        ws = workspace(count, g1.device.index)
    assert ws.numel() >= lib().hbrbc_pairing_workspace_size(count)
    _check(lib().hbrbc_pairing_check_prepared(g1.data_ptr(), prep.data_ptr(), points,
                                              idx_b.data_ptr(), idx_d.data_ptr(), count,
                                              ok.data_ptr(), ws.data_ptr(),
                                              _stream(g1.device, stream)))
    return ok


def g1_prepare(g1, stream=None):
    """Decode and check G1 points (uint8 [n, 96]) once -- hbbft's public key
    shares pk_i, which the crate holds as curve points and does not decode per
    share.  Returns the device table (uint8) for pairing_check_prepared_keys."""
    torch = _torch()
    n = g1.shape[0]
    assert g1.shape == (n, G1_BYTES) and g1.is_contiguous()
    keys = torch.empty(max(1, lib().hbrbc_g1_prepared_size(n)), dtype=torch.uint8,
                       device=g1.device)
    _check(lib().hbrbc_g1_prepare(g1.data_ptr(), n, keys.data_ptr(), _stream(g1.device, stream)))
    return keys


def pairing_check_prepared_keys(shares, keys, key_points, idx_c, prep, points, idx_b, idx_d,
                                ws=None, stream=None):
    """count checks e(a_i, P[idx_b[i]]) == e(K[idx_c[i]], P[idx_d[i]]): shares
    uint8 [count, 96] = a_0, a_1, ...; K = `key_points` prepared G1 keys
    (g1_prepare), P = `points` prepared G2 points (g2_prepare); idx_* int32
    [count].  Returns uint8 [count]: 1 equal, 0 not, 2 invalid point or index."""
    torch = _torch()
    count = shares.shape[0]
    assert shares.shape == (count, G1_BYTES) and shares.is_contiguous()
    for t in (idx_b, idx_c, idx_d):
        assert t.shape == (count,) and t.dtype == torch.int32 and t.is_contiguous()
    ok = torch.empty((count,), dtype=torch.uint8, device=shares.device)
    if ws is None:
        ws = workspace(count, shares.device.index)
    assert ws.numel() >= lib().hbrbc_pairing_workspace_size(count)
    _check(lib().hbrbc_pairing_check_prepared_keys(
        shares.data_ptr(), keys.data_ptr(), key_points, idx_c.data_ptr(), prep.data_ptr(), points,
        idx_b.data_ptr(), idx_d.data_ptr(), count, ok.data_ptr(), ws.data_ptr(),
        _stream(shares.device, stream)))
    return ok


def pairing_check_prepared_pts(a_prep, count, keys, key_points, idx_c, prep, points, idx_b, idx_d,
                               ws=None, stream=None):
    """pairing_check_prepared_keys with the shares decoded beforehand:
    a_prep = g1_prepare(shares) over the `count` shares (a_i = entry i), so
    their decoding can run as its own launch (e.g. beside g2_prepare on
    another stream).  Returns uint8 [count] as pairing_check_prepared_keys."""
    torch = _torch()
    for t in (idx_b, idx_c, idx_d):
        assert t.shape == (count,) and t.dtype == torch.int32 and t.is_contiguous()
    assert a_prep.numel() >= lib().hbrbc_g1_prepared_size(count)
    ok = torch.empty((count,), dtype=torch.uint8, device=a_prep.device)
    if ws is None:
        ws = workspace(count, a_prep.device.index)
    assert ws.numel() >= lib().hbrbc_pairing_workspace_size(count)
    _check(lib().hbrbc_pairing_check_prepared_pts(
        a_prep.data_ptr(), keys.data_ptr(), key_points, idx_c.data_ptr(), prep.data_ptr(), points,
        idx_b.data_ptr(), idx_d.data_ptr(), count, ok.data_ptr(), ws.data_ptr(),
        _stream(a_prep.device, stream)))
    return ok


def verify_decryption_shares_grouped(ciphertexts, shares, device=0):
    """`verify_decryption_share` for many shares of a few ciphertexts, as
    ThresholdDecrypt receives them: ciphertexts = [(hash G2, W G2)], shares =
    [(ciphertext index, share G1, pk_share G1)].  Each ciphertext's H and W
    are prepared once, each distinct key share pk_i is decoded and checked
    once (the crate holds the validator set's key shares as points), the
    received shares are decoded in a launch of their own; shares are grouped
    by ciphertext so a wave shares its lines.  Returns bools in the order of
    `shares`."""
    import numpy as np
    torch = _torch()
    if not shares:
        return []
    dev = "cuda:%d" % device
    g2 = np.empty((2 * len(ciphertexts), G2_BYTES), np.uint8)
    for j, (h, w) in enumerate(ciphertexts):
        g2[2 * j] = np.frombuffer(h, np.uint8)
        g2[2 * j + 1] = np.frombuffer(w, np.uint8)
    key_ids = {}
    for _, _, pk in shares:
        key_ids.setdefault(bytes(pk), len(key_ids))
    kt = np.stack([np.frombuffer(k, np.uint8) for k in key_ids])
    order = sorted(range(len(shares)), key=lambda i: shares[i][0])
    g1 = np.empty((len(shares), G1_BYTES), np.uint8)
    ib = np.empty(len(shares), np.int32)
    ic = np.empty(len(shares), np.int32)
    for r, i in enumerate(order):
        ct, share, pk = shares[i]
        g1[r] = np.frombuffer(share, np.uint8)
        ib[r] = 2 * ct
        ic[r] = key_ids[bytes(pk)]
    d2, dk, d1 = (torch.from_numpy(x).to(dev) for x in (g2, kt, g1))
    # the three preparations are independent: the G2 points and the key
    # shares are latency-bound chains on few waves, the received shares fill
    # the chip -- each on a stream of its own, the checks wait for all three
    cur = torch.cuda.current_stream(dev)
    sides = [torch.cuda.Stream(dev) for _ in range(3)]
    for s_ in sides:
        s_.wait_stream(cur)
    with torch.cuda.stream(sides[0]):
        prep = g2_prepare(d2)
    with torch.cuda.stream(sides[1]):
        ktab = g1_prepare(dk)
    with torch.cuda.stream(sides[2]):
        sprep = g1_prepare(d1)
    for s_ in sides:
        cur.wait_stream(s_)
    for t_, s_ in ((d2, sides[0]), (dk, sides[1]), (d1, sides[2])):
        t_.record_stream(s_)
    for t_ in (prep, ktab, sprep):
        t_.record_stream(cur)
    ok = pairing_check_prepared_pts(sprep, len(shares), ktab, len(key_ids),
                                    torch.from_numpy(ic).to(dev), prep, 2 * len(ciphertexts),
                                    torch.from_numpy(ib).to(dev), torch.from_numpy(ib + 1).to(dev))
    okh = ok.cpu().tolist()
    out = [False] * len(shares)
    for r, i in enumerate(order):
        out[i] = okh[r] == CHECK_OK
    return out


def pairing_check(a, b, c, d):
    """Per-call shim: e(a, b) == e(c, d) for host byte strings (one device
    round trip).  Raises RseError(InvalidArgument) on an invalid point."""
    for x, n in ((a, G1_BYTES), (b, G2_BYTES), (c, G1_BYTES), (d, G2_BYTES)):
        if len(x) != n:
            raise ValueError("point encoding of %d bytes, expected %d" % (len(x), n))
    res = ctypes.c_int(0)
    _check(lib().hbrbc_pairing_check(bytes(a), bytes(b), bytes(c), bytes(d), ctypes.byref(res)))
    return bool(res.value)


def _pack(items, device):
    """[(a, b, c, d)] host bytes -> (g1 [2n, 96], g2 [2n, 192]) on `device`."""
    import numpy as np
    torch = _torch()
    n = len(items)
    g1 = np.empty((2 * n, G1_BYTES), dtype=np.uint8)
    g2 = np.empty((2 * n, G2_BYTES), dtype=np.uint8)
    for i, (a, b, c, d) in enumerate(items):
        g1[2 * i] = np.frombuffer(a, np.uint8)
        g1[2 * i + 1] = np.frombuffer(c, np.uint8)
        g2[2 * i] = np.frombuffer(b, np.uint8)
        g2[2 * i + 1] = np.frombuffer(d, np.uint8)
    dev = "cuda:%d" % device
    return torch.from_numpy(g1).to(dev), torch.from_numpy(g2).to(dev)


def verify_decryption_shares(items, device=0):
    """Batched `PublicKeyShare::verify_decryption_share` (threshold_decrypt.rs:
    220-228): items = [(share G1, pk_share G1, hash G2, W G2)] host bytes.
    Returns a list of bools (an invalid point is False, as a share that does
    not deserialise never reaches the check)."""
    if not items:
        return []
    g1, g2 = _pack([(s, h, pk, w) for s, pk, h, w in items], device)
    ok = pairing_check_batch(g1, g2).cpu().tolist()
    return [v == CHECK_OK for v in ok]


def verify_ciphertexts(items, device=0):
    """Batched `Ciphertext::verify` (threshold_decrypt.rs:142): items =
    [(U G1, W G2, hash G2)]; e(G1::one(), W) == e(U, hash)."""
    if not items:
        return []
    g1, g2 = _pack([(G1_ONE, w, u, h) for u, w, h in items], device)
    ok = pairing_check_batch(g1, g2).cpu().tolist()
    return [v == CHECK_OK for v in ok]
