"""Provenance of libhbrbc.so: a hash of the sources it is built from.

The Makefile (hbbft_amd/csrc/Makefile) runs this file and compiles the hash
into the library (`hbrbc_version()` ends in "src=<hash>"); smoke() and
tests/test_abi.py recompute it from the tree they run from and require the
two to agree, so a prebuilt library that does not match its sources fails
loudly instead of being tested in their place.

Hashed: every *.hip / *.hpp / *.cpp / *.h file and the Makefile of
hbbft_amd/csrc, and every header of include/, by relative path and content,
in sorted path order.  No third-party imports (make runs it with bare python3).
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root=ROOT):
    out = []
    for sub, keep in (("hbbft_amd/csrc", (".hip", ".hpp", ".cpp", ".h")),
                      ("include", (".h", ".hpp"))):
        d = os.path.join(root, sub)
        for name in os.listdir(d):
            if name.endswith(keep) or (sub == "hbbft_amd/csrc" and name == "Makefile"):
                out.append(sub + "/" + name)
    return sorted(out)


def source_hash(root=ROOT):
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            data = f.read()
        h.update(len(data).to_bytes(8, "little") + data)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash(sys.argv[1] if len(sys.argv) > 1 else ROOT))
