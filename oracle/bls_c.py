"""ctypes wrapper for oracle/libbls.so (bls_pairing.c, the C restatement of
the BLS12-381 pairing check).  TEST INFRASTRUCTURE ONLY: used by tests/ and
bench.py's f4 cpu_baseline leg, never by the product path."""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "libbls.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(_PATH)
        L.bls_c_pairing.restype = ctypes.c_int
        L.bls_c_pairing.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.bls_c_check.restype = ctypes.c_int
        L.bls_c_check.argtypes = [ctypes.c_char_p] * 4
        L.bls_c_check_batch.restype = None
        L.bls_c_check_batch.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_int]
        L.bls_c_pairing_batch.restype = None
        L.bls_c_pairing_batch.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def pairing(g1, g2):
    """(576 GT bytes, status 0 ok / 2 invalid) of e(g1, g2), uncompressed encodings."""
    out = ctypes.create_string_buffer(576)
    st = lib().bls_c_pairing(bytes(g1), bytes(g2), out)
    return out.raw, st


def check(a, b, c, d):
    """1 if e(a, b) == e(c, d), 0 if not, 2 if a point is invalid."""
    return lib().bls_c_check(bytes(a), bytes(b), bytes(c), bytes(d))


def check_batch(g1, g2, count, threads):
    """hbrbc_pairing_check_batch's layout (g1: a_i, c_i; g2: b_i, d_i) as bytes;
    returns a bytes object of count outcomes."""
    ok = ctypes.create_string_buffer(count)
    lib().bls_c_check_batch(bytes(g1), bytes(g2), count, ok, threads)
    return ok.raw


def pairing_batch(g1, g2, count, threads):
    """count pairings (uncompressed encodings, concatenated) -> (gt bytes
    [count * 576], status bytes [count])."""
    gt = ctypes.create_string_buffer(576 * count)
    st = ctypes.create_string_buffer(count)
    lib().bls_c_pairing_batch(bytes(g1), bytes(g2), count, gt, st, threads)
    return gt.raw, st.raw
