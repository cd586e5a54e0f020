// Source stamp of libbcg_kernels.so: utils/build.py passes a hash of every
// csrc/kernels/*.hip / *.h file as BCG_SOURCE_HASH, and ops/hip.py refuses a
// library whose stamp differs from the tree it is loaded from (a stale binary
// shipped next to newer sources must never run).
#include "common.h"

#ifndef BCG_SOURCE_HASH
#define BCG_SOURCE_HASH "unstamped"
#endif

BCG_API const char* bcg_source_hash() { return BCG_SOURCE_HASH; }
