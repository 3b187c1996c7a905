// Build provenance of libcosnet_hip.so: the SHA-256 (first 16 hex digits) of the HIP sources
// and the C-ABI header it was compiled from, stamped in by the Makefile (CN_SRC_HASH), so a
// caller can check that the library it loaded was built from the sources it ships with
// (bench.py records both hashes in its JSON line).
#include "../../include/cosnet_hip.h"
#include "common.h"

#ifndef CN_SRC_HASH
#define CN_SRC_HASH "unknown"
#endif

extern "C" const char* cn_build_source_hash(void) { return CN_SRC_HASH; }

extern "C" int cn_build_experimental(void) { return CN_EXPERIMENTAL; }
