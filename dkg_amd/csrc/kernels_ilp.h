// The dkgk_ilp copy of the kernel launchers: kernels.hip compiled a second time with DKG_FE_ILP
// (the column-sum field multiplication of fe25519.h: more independent mad chains per multiply,
// for launches whose SIMDs hold too few waves to hide product scanning's serial chain).  Same
// signatures and semantics as kernels.h; the runtime picks the copy per launch (DESIGN.md
// section 5).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define dkgk dkgk_ilp
#include "kernels_decl.inc"
#undef dkgk
