// hbrbc_version(): the library's version plus the hash of the sources it was
// built from (hbbft_amd/srchash.py, passed in by the Makefile), so a GPU-side
// record can show which tree a prebuilt libhbrbc.so came from.
#include "../../include/hbrbc.h"

#ifndef HBRBC_SRC_HASH
#error "HBRBC_SRC_HASH must be defined by the Makefile (python3 ../srchash.py)"
#endif

extern "C" const char *hbrbc_version(void) { return "hbrbc 0.3.0 gfx950 src=" HBRBC_SRC_HASH; }
