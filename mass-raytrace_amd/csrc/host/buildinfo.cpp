// buildinfo.cpp — mrt_build_info(): the source hash this library was built
// from (tools/src_hash.py, written to $(BUILD)/src_hash.h by the Makefile).
#include "../../../include/massrt.h"
#include "src_hash.h"

extern "C" const char* mrt_build_info(void) { return "src " MRT_SRC_HASH; }
