// jit.hip — the step kernels specialised for ONE model at run time (mjlab_amd/jit.py): the
// same kernel source as spec.hip, compiled by hipcc when a Simulation's model matches no
// csrc/specs.inc entry, into a small shared library that libmjx355 loads and registers
// (mjx_spec_register).  Set by the build: MJX_SPECS_FILE (a generated specs file holding the
// entry) and MJX_JIT_ID (its id: distinct per entry, so that no template instantiation
// shares a name with the main library's or another JIT library's; built with
// -fvisibility=hidden, only the three entry points below are exported).
#include "engine_impl.h"

#ifndef MJX_JIT_ID
#error "MJX_JIT_ID must name the generated entry"
#endif

namespace mjx {
static_assert(ModelSpec<MJX_JIT_ID>::on, "the generated specs file lacks the entry");
}  // namespace mjx

#ifndef MJX_HDR_HASH
#error "MJX_HDR_HASH must be the kernel-header hash (mjlab_amd/jit.py, csrc/Makefile)"
#endif
extern "C" __attribute__((visibility("default"))) int mjx_jit_abi(void) { return (int)sizeof(mjx::Dims); }
// the kernel headers this library was compiled from (must equal libmjx355's own)
extern "C" __attribute__((visibility("default"))) unsigned long long mjx_jit_hdr(void) {
  return MJX_HDR_HASH;
}
extern "C" __attribute__((visibility("default"))) void mjx_jit_dims(mjx::Dims* out) {
  *out = mjx::ModelSpec<MJX_JIT_ID>::dims();
}
extern "C" __attribute__((visibility("default"))) int mjx_jit_tree(int* par, int cap) {
  const int n = mjx::SpecTree<MJX_JIT_ID>::npar;
  for (int i = 0; i < n && i < cap; i++) par[i] = mjx::SpecTree<MJX_JIT_ID>::par[i];
  return n;
}
extern "C" __attribute__((visibility("default"))) mjx::StepFn mjx_jit_kernel(int ph) {
  return mjx::phase_kernel<mjx::spec_nr<MJX_JIT_ID>(), MJX_JIT_ID>(ph);
}
