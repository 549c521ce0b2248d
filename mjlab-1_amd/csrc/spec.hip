// spec.hip — the step kernels compiled for ONE model specialisation (specs.inc entry
// MJX_SPEC_ID, set by the Makefile): same kernel source as the generic build
// (engine_impl.h), with every dimension and LDS carve offset a compile-time constant.
#include "engine_impl.h"

#ifndef MJX_SPEC_ID
#error "MJX_SPEC_ID must name a specs.inc entry"
#endif

namespace mjx {

#define MJX_CAT2(a, b) a##b
#define MJX_CAT(a, b) MJX_CAT2(a, b)
StepFn MJX_CAT(spec_fn_, MJX_SPEC_ID)(int ph) {
  constexpr int NR = spec_nr<MJX_SPEC_ID>();
  static_assert(ModelSpec<MJX_SPEC_ID>::on, "unknown specialisation");
  // ph 3: the latency form of phase B (full-capacity row class, masked forward); 4-6: the
  // overflow re-solve's A / B / C (phase_kernel)
  return phase_kernel<NR, MJX_SPEC_ID>(ph);
}

}  // namespace mjx
