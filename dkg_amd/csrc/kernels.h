// Host-side launchers for the gfx950 kernels (kernels.hip).  All pointers are device pointers;
// all launches go to `stream`.  Layouts are documented in points.h and DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "kernels_decl.inc"

