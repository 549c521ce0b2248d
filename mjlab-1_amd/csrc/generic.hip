// generic.hip — the generic step kernels (dims read at run time) for ONE register-row length
// NR (MJX_GENERIC_NR, set by the Makefile: 8 16 20 24 32 36 40 48 56 64).  One object per NR
// so that the instantiations compile in parallel (make -j); engine.hip picks by nv.
#include "engine_impl.h"

#ifndef MJX_GENERIC_NR
#error "MJX_GENERIC_NR must be set"
#endif

namespace mjx {

#define MJX_CAT2(a, b) a##b
#define MJX_CAT(a, b) MJX_CAT2(a, b)
StepFn MJX_CAT(generic_fn_, MJX_GENERIC_NR)(int ph) { return phase_kernel<MJX_GENERIC_NR, 0>(ph); }

}  // namespace mjx
