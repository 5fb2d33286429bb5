// The source hash this library was built from (Makefile: SMMD_SRC_HASH), so the
// Python binding can refuse a stale binary whose sources have since changed.
#include "smmd_hip.h"

#ifndef SMMD_SRC_HASH
#error "build through the Makefile: it passes -DSMMD_SRC_HASH"
#endif

extern "C" const char *smmd_source_hash(void) { return SMMD_SRC_HASH; }
