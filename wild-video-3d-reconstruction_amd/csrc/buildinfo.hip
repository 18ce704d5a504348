// buildinfo.hip -- build provenance of libdpvo_hot.so (include/dpvo_hot.h,
// dpvo_hot_build_info).  DPVO_SRC_SHA is set by the Makefile from the sources
// it compiles; this object is rebuilt on every make.
#include "common.hpp"

#ifndef DPVO_SRC_SHA
#error "DPVO_SRC_SHA must be defined by the build (see Makefile)"
#endif
#if defined(DPVO_EXP_FLAVOUR)
#define DPVO_FLAVOUR DPVO_EXP_FLAVOUR   // experiment builds (scripts/build_exp.sh): refused unless DPVO_DIAG=1
#elif defined(DPVO_STAMPS)
#define DPVO_FLAVOUR "stamps"
#else
#define DPVO_FLAVOUR "product"
#endif

extern "C" const char* dpvo_hot_build_info(void) { return "sha=" DPVO_SRC_SHA " flavour=" DPVO_FLAVOUR; }
