// engine.hip — host side of the mjx355 step engine for MI355X (gfx950): the generic step
// kernels (any model, dims read at run time), the reset kernel, kernel selection
// (generic vs model-specialised, specs.inc) and the launchers.  The kernels themselves are
// in engine_impl.h; spec.hip compiles them once per specs.inc entry.
#include "engine_impl.h"

#include <vector>

namespace mjx {

// --------------------------------------------------------------------------- reset
__global__ void reset_kernel(Dims d, DModel m, DData D, const uint8_t* mask, int nworld,
                             int con_stride) {
  const int w = blockIdx.x;
  if (w >= nworld) return;
  if (mask && !mask[w]) return;
  const int lane = threadIdx.x;
  const float* qpos0 = m.qpos0 + (size_t)w * m.qpos0_ws;
  for (int i = lane; i < d.nq; i += blockDim.x) D.qpos[(size_t)w * d.nq + i] = qpos0[i];
  for (int i = lane; i < d.nv; i += blockDim.x) {
    size_t k = (size_t)w * d.nv + i;
    D.qvel[k] = 0; D.qacc_warmstart[k] = 0; D.qacc[k] = 0; D.qfrc_applied[k] = 0;
    D.qacc_smooth[k] = 0; D.qfrc_constraint[k] = 0;
  }
  for (int i = lane; i < d.nu; i += blockDim.x) {
    D.ctrl[(size_t)w * d.nu + i] = 0; D.actuator_force[(size_t)w * d.nu + i] = 0;
  }
  for (int i = lane; i < 6 * d.nbody; i += blockDim.x) D.xfrc_applied[(size_t)w * 6 * d.nbody + i] = 0;
  for (int i = lane; i < d.nsensordata; i += blockDim.x) D.sensordata[(size_t)w * d.nsensordata + i] = 0;
  for (int b = lane; b < d.nbody; b += blockDim.x) {
    int mid = m.body_mocapid[b];
    if (mid < 0) continue;
    const float* bp = m.body_pos + (size_t)w * m.body_pos_ws + 3 * b;
    const float* bq = m.body_quat + (size_t)w * m.body_quat_ws + 4 * b;
    for (int t = 0; t < 3; t++) D.mocap_pos[((size_t)w * d.nmocap + mid) * 3 + t] = bp[t];
    for (int t = 0; t < 4; t++) D.mocap_quat[((size_t)w * d.nmocap + mid) * 4 + t] = bq[t];
  }
  // contact output slots (mj_resetData: no contacts) up to the last output's reach, and the
  // output bookkeeping of engine_counters [6] / [7] with them (phase A's output trims to it)
  int* wsv = D.wstats + 8 * (size_t)w;
  const int nout = min(con_stride, max(wsv[6], wsv[7]));
  const size_t wc = (size_t)w * con_stride;
  for (int c = lane; c < nout; c += blockDim.x) {
    D.contact_dist[wc + c] = 0.f;
    D.contact_geom[(wc + c) * 2] = -1;
    D.contact_geom[(wc + c) * 2 + 1] = -1;
    for (int t = 0; t < 3; t++) D.contact_pos[(wc + c) * 3 + t] = 0.f;
    for (int t = 0; t < 9; t++) D.contact_frame[(wc + c) * 9 + t] = 0.f;
    for (int t = 0; t < 3; t++) D.contact_force[(wc + c) * 3 + t] = 0.f;
  }
  __syncthreads();
  if (lane == 0) { D.time[w] = 0; D.ncon[w] = 0; D.nefc[w] = 0; wsv[6] = 0; wsv[7] = 0; }
}

// ------------------------------------------------------------------ Newton work lists
// One workgroup: counting sort of the worlds by constraint-row count (phase A's D.nefc),
// descending, then the segment of each row class.  Worlds outside `mask` are not listed.
// Order within equal row counts follows LDS atomics (each world's result is independent of
// it).
constexpr int kClassifyThreads = 1024;
constexpr int kMaxRowBins = 2048;
__global__ __launch_bounds__(kClassifyThreads) void classify_kernel(const Params* __restrict__ P,
                                                                    int w0, int w1, int split,
                                                                    const uint8_t* __restrict__ mask) {
  __shared__ int bin[kMaxRowBins];
  __shared__ int wsum[kClassifyThreads / kWave];
  constexpr int nwave = kClassifyThreads / kWave;
  const int nb = min(P->d.njmax + 1, kMaxRowBins);
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  for (int i = t; i < nb; i += kClassifyThreads) bin[i] = 0;
  __syncthreads();
  const int* nefc = P->D.nefc;
  // worlds listed for the overflow re-solve this substep (phase A left nefc = -1) are not
  // classed: the max launch set solves them
  for (int w = w0 + t; w < w1; w += kClassifyThreads) {
    const int r = nefc[w];
    if ((!mask || mask[w]) && r >= 0) atomicAdd(&bin[min(r, nb - 1)], 1);
  }
  __syncthreads();
  // exclusive scan of the bins in descending row count: bin[r] <- #listed worlds with more
  // than r rows.  Thread t owns a contiguous chunk of the reversed bin order.
  const int per = (nb + kClassifyThreads - 1) / kClassifyThreads;
  const int i0 = min(t * per, nb), i1 = min(i0 + per, nb);
  int run = 0;
  for (int i = i0; i < i1; i++) run += bin[nb - 1 - i];
  int x = run;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) wsum[wv] = x;
  __syncthreads();
  if (wv == 0) {
    int v = lane < nwave ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(v, o);
      if (lane >= o) v += y;
    }
    if (lane < nwave) wsum[lane] = v;  // inclusive over waves
  }
  __syncthreads();
  const int total = wsum[nwave - 1];
  int base = x - run + (wv > 0 ? wsum[wv - 1] : 0);
  for (int i = i0; i < i1; i++) {
    const int r = nb - 1 - i, c = bin[r];
    bin[r] = base;
    base += c;
  }
  __syncthreads();
  // row class k's segment: class 0 = rows > cap[nc-1] (the front of the list), class k >= 1
  // = rows in (cap[k-2], cap[k-1]] (class 1 from 0 rows)
  const int nc = P->nrowclass;
  if (t <= nc) {
    const int hi = t == 0 ? nb - 1 : min(P->row_cap[t - 1], nb - 1);
    const int lo = t == 0 ? (nc > 0 ? P->row_cap[nc - 1] : -1) : (t > 1 ? P->row_cap[t - 2] : -1);
    const int s0 = bin[hi];
    const int s1 = lo < 0 ? total : bin[min(lo, nb - 1)];
    // this split's list occupies wl_list[w0, w1): absolute segment starts
    int* seg = P->wl_seg + 2 * (kRowClasses + 1) * split;
    seg[2 * t] = w0 + s0;
    seg[2 * t + 1] = max(s1 - s0, 0);
  }
  __syncthreads();  // the segments read the bins before the scatter advances them
  for (int w = w0 + t; w < w1; w += kClassifyThreads) {
    const int r = nefc[w];
    if ((!mask || mask[w]) && r >= 0) P->wl_list[w0 + atomicAdd(&bin[min(r, nb - 1)], 1)] = w;
  }
}

// Generic kernels: one instantiation per (register-row length NR >= padded nv; phase), each
// NR in its own object (generic.hip with -DMJX_GENERIC_NR, compiled in parallel).
#define MJX_GENERIC_NRS(X) X(8) X(16) X(20) X(24) X(32) X(36) X(40) X(48) X(56) X(64)
#define MJX_DECL_GENERIC(nr) StepFn generic_fn_##nr(int ph);
MJX_GENERIC_NRS(MJX_DECL_GENERIC)
#undef MJX_DECL_GENERIC
static StepFn generic_fn(int nv, int ph) {
  // exact fits for the shipped robots (Go1 nvp 20, G1 nvp 36), multiples of 8 otherwise
  const int nvp = (nv + 3) & ~3;
  if (nvp <= 8) return generic_fn_8(ph);
  if (nvp <= 16) return generic_fn_16(ph);
  if (nvp <= 20) return generic_fn_20(ph);
  if (nvp <= 24) return generic_fn_24(ph);
  if (nvp <= 32) return generic_fn_32(ph);
  if (nvp <= 36) return generic_fn_36(ph);
  if (nvp <= 40) return generic_fn_40(ph);
  if (nvp <= 48) return generic_fn_48(ph);
  if (nvp <= 56) return generic_fn_56(ph);
  return generic_fn_64(ph);
}

// Model-specialised kernels (spec.hip, one object per specs.inc entry).
#define MJX_SPEC(id, scene, ...) StepFn spec_fn_##id(int ph);
#include "specs.inc"
#undef MJX_SPEC
// Run-time specialisations (jit.hip libraries, mjx_spec_register): ids kRtSpecBase + i.
struct RtSpec {
  Dims d;
  std::vector<int> par;
  StepFn (*fn)(int);
};
static std::vector<RtSpec>& rt_specs() {
  static std::vector<RtSpec> v;
  return v;
}
int register_spec(const Dims& d, const int* par, int npar, StepFn (*fn)(int)) {
  rt_specs().push_back(RtSpec{d, std::vector<int>(par, par + npar), fn});
  return kRtSpecBase + (int)rt_specs().size() - 1;
}
static StepFn spec_fn(int spec, int ph) {
  if (spec >= kRtSpecBase) {
    const int i = spec - kRtSpecBase;
    return i < (int)rt_specs().size() ? rt_specs()[i].fn(ph) : nullptr;
  }
  switch (spec) {
#define MJX_SPEC(id, scene, ...) case id: return spec_fn_##id(ph);
#include "specs.inc"
#undef MJX_SPEC
    default: return nullptr;
  }
}
static StepFn step_fn(const Params& host, int ph) {
  StepFn f = host.spec > 0 ? spec_fn(host.spec, ph) : nullptr;
  return f ? f : generic_fn(host.d.nv, ph);
}
// The full-capacity Newton class and the masked forward run the latency kernel
// (step_newton_lat); MJX355_NEWTON_LAT=0 keeps them on step_phase<NR, 1> (A/B diagnostic).
static bool newton_lat() {
  static const bool on = [] {
    const char* e = getenv("MJX355_NEWTON_LAT");
    return !e || atoi(e) != 0;
  }();
  return on;
}
// The full-capacity class's latency Newton kernel at the throughput kernels' 168 VGPRs (phase
// code 12; naturally ~193, 68 B per lane spilled when capped), its waves at raised issue
// priority (kSelPrio): a SIMD running a heavy world keeps two bulk-class waves beside it instead
// of one, and the heavy wave still issues first.  Measured (three interleaved rounds on one
// box): G1 velocity 4,096 +0.4 / +0.7 / +1.2 %, rough G1 +0.4 / +0.2 / +0.8 %; tracking (its
// 56 / 200 carve, heavy worlds up to ~190 rows) -0.7 / -0.3 / -0.6 %: on for fast carves of at
// most 160 rows.  MJX355_HEAVY_CAP=0/1 forces.
static bool heavy_cap(const Params& host) {
  static const int mode = [] {
    const char* e = getenv("MJX355_HEAVY_CAP");
    return e ? atoi(e) : -1;
  }();
  return mode >= 0 ? mode != 0 : host.d.njmax <= 160;
}
// The full-capacity row class (the heavy worlds of the fast carve) reads the constraint
// Jacobian from the B pack in global memory (carve kLdsJG) instead of an LDS copy.
// MJX355_NEWTON_JG (A/B): 0 off, 1 the latency kernel (phase code 9), 2 the throughput kernel
// (phase code 10); with MJX355_CHAIN covering the full-capacity class, its chain (code 11).
static int newton_jg() {
  static const int mode = [] {
    const char* e = getenv("MJX355_NEWTON_JG");
    return e ? atoi(e) : -1;
  }();
  return mode;
}

int find_spec(const Dims& d, const int* dof_parentid) {
  if (const char* e = getenv("MJX355_NO_SPEC"))  // diagnostic: force the generic kernels
    if (atoi(e) != 0) return 0;
  auto eq = [](const Dims& a, const Dims& b) {
    return a.nq == b.nq && a.nv == b.nv && a.nu == b.nu && a.nbody == b.nbody &&
           a.njnt == b.njnt && a.ngeom == b.ngeom && a.nsite == b.nsite &&
           a.nsensor == b.nsensor && a.nsensordata == b.nsensordata && a.npair == b.npair &&
           a.nhfield == b.nhfield && a.nhfielddata == b.nhfielddata && a.nlevel == b.nlevel &&
           a.nchild == b.nchild && a.nmocap == b.nmocap && a.ngeom_lds == b.ngeom_lds &&
           a.npair_all == b.npair_all && a.nstatic == b.nstatic &&
           a.nstpartner == b.nstpartner && a.nboxbox == b.nboxbox && a.nconmax == b.nconmax && a.njmax == b.njmax;
  };
  // and the dof tree of the entry's tree-form SPD factors (rows_chol_tree)
  auto same_tree = [&](const int* par, int n) {
    if (n != d.nv) return false;
    for (int i = 0; i < n; i++)
      if (dof_parentid[i] != par[i]) return false;
    return true;
  };
#define MJX_SPEC(id, scene, ...) \
  if (eq(d, ModelSpec<id>::dims()) && same_tree(SpecTree<id>::par, SpecTree<id>::npar)) return id;
#include "specs.inc"
#undef MJX_SPEC
  for (int i = 0; i < (int)rt_specs().size(); i++) {
    const RtSpec& r = rt_specs()[i];
    if (eq(d, r.d) && same_tree(r.par.data(), (int)r.par.size())) return kRtSpecBase + i;
  }
  return 0;
}

// Diagnostic: MJX355_LDS_PAD=<bytes> (all phases) or MJX355_LDS_PAD<ph>=<bytes> (phase 0/1/2)
// adds unused dynamic LDS per world, to measure how throughput depends on resident worlds
// per CU.
static size_t lds_bytes(const Params& host, int ph) {
  static const long pad[3] = {[] { const char* e = getenv("MJX355_LDS_PAD0"); return e ? atol(e) : 0L; }(),
                              [] { const char* e = getenv("MJX355_LDS_PAD1"); return e ? atol(e) : 0L; }(),
                              [] { const char* e = getenv("MJX355_LDS_PAD2"); return e ? atol(e) : 0L; }()};
  static const long pad_all = [] {
    const char* e = getenv("MJX355_LDS_PAD");
    return e ? atol(e) : 0L;
  }();
  const long p = pad_all + pad[ph >= 3 ? 1 : ph];
  const Lds& L = ph == kLdsJG ? host.LPJ : host.LP[ph];
  return (size_t)L.total * 4 + (size_t)(p > 0 ? p : 0);
}

// dynamic LDS of step_resolve: the largest of the three phase carves
static size_t lds_resolve(const Params& host) {
  return std::max(lds_bytes(host, 0), std::max(lds_bytes(host, 1), lds_bytes(host, 2)));
}
// dynamic LDS of a class chain (step_chain): the class's Newton carve, phase C's and, when it
// runs the next phase A, phase A's
static size_t lds_chain(const Params& host, int cls, bool with_a, bool jg = false) {
  size_t b = std::max(lds_bytes(host, cls ? 2 + cls : jg ? kLdsJG : 1), lds_bytes(host, 2));
  return with_a ? std::max(b, lds_bytes(host, 0)) : b;
}
// Which class chains run as one launch (step_chain).  Default: the bulk class (the fewest
// rows, most worlds, on the launch stream) when the batch is at most kChainMaxWorlds.
// Measured (G1 4,096, two interleaved rounds on one box): bulk chained 2.81 M env-steps/s,
// every class chained 2.70 M, none 2.67 M, only the heavy classes 2.58 M -- the heavy class's
// latency kernel then runs its C and next A at one wave per SIMD; jump hfield at 16,384
// worlds (five residency rounds, whose per-slot sums already average the Newton tails):
// none 4.54 M, bulk 4.52 M, all 4.44 M.  MJX355_CHAIN (A/B diagnostic): 0 none, 1 every
// class, 2 the bulk class at any batch size, 3 only the others.
constexpr int kChainMaxWorlds = 8192;
// J-in-global mode of the full-capacity class (newton_jg): by default the throughput form past
// kChainMaxWorlds worlds, where that class holds thousands of worlds and its launch is
// throughput-bound by its LDS carve (jump hfield 16,384: ~5,400 worlds at 84-137 rows, 4 per CU
// with J in LDS, 12 per CU without; 4.64 -> 4.80 M env-steps/s, two interleaved rounds), and
// off below (G1 4,096: ~670 heavy worlds, one per SIMD at most: +-0.5 %; tracking -1 %)
static int jg_mode(int nworld) {
  const int m = newton_jg();
  return m >= 0 ? m : nworld > kChainMaxWorlds ? 2 : 0;
}
static bool chain_env(int cls, int nworld) {
  static const int mode = [] {
    const char* e = getenv("MJX355_CHAIN");
    return e ? atoi(e) : -1;
  }();
  if (mode < 0) return cls == 1 && nworld <= kChainMaxWorlds;
  return mode == 1 || (mode == 2 && cls == 1) || (mode == 3 && cls != 1);
}

hipError_t prepare_step(const Params& host) {
  size_t shmem[3] = {lds_bytes(host, 0), lds_bytes(host, 1), lds_bytes(host, 2)};
  for (int k = 0; k < host.nrowclass; k++) shmem[1] = std::max(shmem[1], lds_bytes(host, 3 + k));
  for (int ph = 0; ph < 9; ph++) {  // phase codes of phase_kernel
    const size_t need = ph >= 5 ? std::max(shmem[0], std::max(shmem[1], shmem[2]))
                                : shmem[ph == 3 ? 1 : ph == 4 ? 0 : ph];
    const StepFn f = step_fn(host, ph);
    if (need > 64 * 1024 && f) {
      hipError_t e = hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)need);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// Batch split together with Newton row classes: every fork starts from the launch stream
// and every side stream joins back into it before the next fork ("flat" fork / join).  Per
// substep: [A of each split, classify] on the split streams, join; [each split's class
// chains (B, and piped C + next A) on the class streams, the smallest class on the split
// stream], join.  A fork from one side stream to another (split stream -> its class
// streams, the natural nesting) crashes hipStreamEndCapture under the HIP runtime torch
// bundles (a synthetic probe with no engine code reproduces it in a torch process and not
// standalone on ROCm 7.2: scripts/capture_probe*.{hip,py}), and the
// flat form keeps the capture to the fork / join shape the unsplit class path uses.
static hipError_t launch_split_classes(const Params& host, const Params* dev, int nworld,
                                       int nsubstep, int integrate, hipStream_t stream,
                                       const SideStream* side, int nsplit, bool piped) {
  const StepFn fA = step_fn(host, 0), fB = step_fn(host, 1), fC = step_fn(host, 2);
  const StepFn fBL = newton_lat() ? step_fn(host, 3) : fB;
  const int nc = host.nrowclass;
  hipStream_t sst[kMaxSplit];
  int wb[kMaxSplit + 1];
  for (int k = 0; k <= nsplit; k++) wb[k] = (int)(((long long)nworld * k) / nsplit);
  sst[0] = stream;
  for (int k = 1; k < nsplit; k++) sst[k] = side->split[k];
  hipError_t e = hipSuccess;
  auto fork_all = [&](bool classes) {
    e = hipEventRecord(side->split_fork, stream);
    for (int k = 1; k < nsplit && e == hipSuccess; k++) e = hipStreamWaitEvent(sst[k], side->split_fork, 0);
    for (int k = 0; k < nsplit && classes; k++)
      for (int c = 0; c < nc && e == hipSuccess; c++)
        e = hipStreamWaitEvent(side->stream[k][c], side->split_fork, 0);
    return e;
  };
  auto join_all = [&](bool classes) {
    for (int k = 0; k < nsplit && classes; k++)
      for (int c = 0; c < nc && e == hipSuccess; c++) {
        e = hipEventRecord(side->join[k][c], side->stream[k][c]);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, side->join[k][c], 0);
      }
    for (int k = 1; k < nsplit && e == hipSuccess; k++) {
      e = hipEventRecord(side->split_join[k], sst[k]);
      if (e == hipSuccess) e = hipStreamWaitEvent(stream, side->split_join[k], 0);
    }
    return e;
  };
  for (int sub = 0; sub < nsubstep; sub++) {
    const int last = sub == nsubstep - 1;
    if (fork_all(false) != hipSuccess) return e;
    for (int k = 0; k < nsplit; k++) {
      const int w0 = wb[k], w1 = wb[k + 1], n = w1 - w0;
      if (n <= 0) continue;
      if (!piped || sub == 0)
        hipLaunchKernelGGL(fA, dim3(n), dim3(kWave), lds_bytes(host, 0), sst[k], dev, w0, w1, k,
                           last, integrate, nullptr);
      hipLaunchKernelGGL(classify_kernel, dim3(1), dim3(kClassifyThreads), 0, sst[k], dev, w0, w1,
                         k, nullptr);
    }
    if (join_all(false) != hipSuccess || fork_all(true) != hipSuccess) return e;
    for (int k = 0; k < nsplit; k++) {
      const int w0 = wb[k], w1 = wb[k + 1], n = w1 - w0;
      if (n <= 0) continue;
      auto class_chain = [&](hipStream_t cs, int cls) {
        hipLaunchKernelGGL(cls ? fB : fBL, dim3(n), dim3(kWave), lds_bytes(host, cls ? 2 + cls : 1), cs, dev,
                           w0, w1, k, last, cls, nullptr);
        if (!piped) return;
        hipLaunchKernelGGL(fC, dim3(n), dim3(kWave), lds_bytes(host, 2), cs, dev, w0, w1,
                           k | (cls + 1) << 8, last, integrate, nullptr);
        if (!last)
          hipLaunchKernelGGL(fA, dim3(n), dim3(kWave), lds_bytes(host, 0), cs, dev, w0, w1,
                             k | (cls + 1) << 8, sub + 1 == nsubstep - 1, integrate, nullptr);
      };
      for (int c = 0; c < nc; c++) class_chain(side->stream[k][c], c == 0 ? 0 : nc + 1 - c);
      class_chain(sst[k], 1);
    }
    if (join_all(true) != hipSuccess) return e;
    if (piped) continue;
    if (fork_all(false) != hipSuccess) return e;
    for (int k = 0; k < nsplit; k++) {
      const int w0 = wb[k], w1 = wb[k + 1], n = w1 - w0;
      if (n > 0)
        hipLaunchKernelGGL(fC, dim3(n), dim3(kWave), lds_bytes(host, 2), sst[k], dev, w0, w1, k,
                           last, integrate, nullptr);
    }
    if (join_all(false) != hipSuccess) return e;
  }
  return hipGetLastError();
}

// Overflow re-solve chain of split k at substep `sub` (parity sub & 1): the listed worlds'
// substep at full capacity (step_resolve: max A, latency Newton, C), then -- when the class
// pipelines carry the next substep's phase A -- that phase A in the normal carve; the last
// of them empties the list on exit.  The grid is fixed (kOvfGrid workgroups, each looping
// over listed worlds); workgroups past the listed count exit at once.
static void ovf_chain(const Params& host, const Params* dev, const Params& hbig, const Params* dbig,
                      hipStream_t cs, int k, int w0, int w1, int sub, int nsubstep, int integrate,
                      bool next_a, bool in_line) {
  const int last = sub == nsubstep - 1;
  const int par = sub & 1;
  // the grid: kOvfGrid on a stream of its own (sized for heavy overflow; an empty list costs
  // the same at 1 or 256 workgroups there), kOvfGridInline where the chain runs in line on
  // the critical path (split batches: 256 max-carve workgroups per launch cost Go1 8 %;
  // engine.h kOvfGridInline);
  // MJX355_OVF_GRID overrides both
  static const int grid_env = [] {
    const char* e = getenv("MJX355_OVF_GRID");
    return e && atoi(e) > 0 ? atoi(e) : 0;
  }();
  const int g = std::min(hbig.ovf_cap, grid_env > 0 ? grid_env : in_line ? kOvfGridInline : kOvfGrid);
  const int sel = k | kSelOvf | (par ? kSelRPar : 0);
  const bool next = next_a && !last;
  hipLaunchKernelGGL(step_fn(hbig, 5), dim3(g), dim3(kWave), lds_resolve(hbig), cs, dbig, w0, w1,
                     sel | (next ? 0 : kSelClr), last, integrate, nullptr);
  if (next)
    hipLaunchKernelGGL(step_fn(host, 4), dim3(g), dim3(kWave), lds_bytes(host, 0), cs, dev, w0, w1,
                       sel | kSelClr | ((sub + 1) & 1 ? kSelAPar : 0), sub + 1 == nsubstep - 1,
                       integrate, nullptr);
}

static bool ovf_stream_env() {
  static const bool on = [] {
    const char* e = getenv("MJX355_OVF_STREAM");
    return e && atoi(e) != 0;
  }();
  return on;
}

// Order of the concurrent branches in a captured graph.  Graph replay (ROCm 7 clr) keeps the
// first child of a fork on the launch queue and starts every further child on a parallel
// queue, whose start and join each wait on a cross-queue signal (kernel trace, G1 4,096:
// classify -> bulk chain 12 us on the parallel queue, 5.5 us in line).  So while capturing,
// the models without row classes capture their critical launch (the range chain, phase B)
// ahead of the re-solve chain's: Go1 flat 8,192 +1.2 %, rough Go1 +0.6 % (two interleaved
// rounds).  The row-class fork keeps its order (the full-capacity class first, on the launch
// queue): bulk chain first measured G1 2.94 -> 2.38 M, tracking 2.71 -> 2.19 M, since the
// full class's long-latency worlds then start behind the bulk chain's and end last.
// MJX355_MAIN_FIRST=0 / 1 forces it off / on.
static bool main_first(hipStream_t st) {
  static const int mode = [] {
    const char* e = getenv("MJX355_MAIN_FIRST");
    return e ? atoi(e) : -1;
  }();
  if (mode >= 0) return mode != 0;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}

hipError_t launch_step(const Params& host, const Params* dev, int nworld, int nsubstep,
                       int integrate, const uint8_t* mask, hipStream_t stream,
                       const SideStream* side, const Params* hbig, const Params* dbig) {
  if (nworld <= 0) return hipSuccess;
  // The masked forward (a few reset worlds): its three launches in the max carve, or in the
  // fast carve with the re-solve in line behind them.  The max-carve grid is the whole batch,
  // and at 64 KiB of LDS per workgroup even the unmasked workgroups dispatch two per CU; the
  // in-line re-solve is a fixed launch on the critical path.  Measured: G1 4,096 worlds max
  // carve +1.1 %, jump hfield 16,384 worlds fast carve +9.5 % (round 6, two interleaved rounds:
  // +14 %); round 6, max carve (fused, step_masked): Go1 8,192 +1.5 %, rough Go1 +2.0 %, jump
  // flat 16,384 +0.8 %.  So the max carve unless a heightfield model has more than 4,096
  // worlds (its reset worlds' phase A at the max carve's 300 contacts is the slow part there).
  // MJX355_MASKED_BIG=0/1 forces.
  static const int masked_big_env = [] {
    const char* e = getenv("MJX355_MASKED_BIG");
    return e ? atoi(e) : -1;
  }();
  const bool masked_big = masked_big_env >= 0 ? masked_big_env != 0 : nworld <= 4096 || host.d.nhfield == 0;
  if (mask && hbig && masked_big) {
    // masked forward (a few reset worlds): at full capacity throughout -- nothing to re-solve;
    // A -> B -> C as one launch (step_masked) unless MJX355_MASKED_FUSED=0
    static const bool fused = [] {
      const char* e = getenv("MJX355_MASKED_FUSED");
      return !e || atoi(e) != 0;
    }();
    if (const StepFn fM = fused ? step_fn(*hbig, 8) : nullptr) {
      hipLaunchKernelGGL(fM, dim3(nworld), dim3(kWave), lds_resolve(*hbig), stream, dbig, 0, nworld, 0,
                         1, integrate, mask);
      return hipGetLastError();
    }
    const StepFn fA = step_fn(*hbig, 0), fBL = step_fn(*hbig, 3), fC = step_fn(*hbig, 2);
    hipLaunchKernelGGL(fA, dim3(nworld), dim3(kWave), lds_bytes(*hbig, 0), stream, dbig, 0, nworld, 0,
                       1, integrate, mask);
    hipLaunchKernelGGL(fBL, dim3(nworld), dim3(kWave), lds_bytes(*hbig, 1), stream, dbig, 0, nworld, 0,
                       1, -1, mask);
    hipLaunchKernelGGL(fC, dim3(nworld), dim3(kWave), lds_bytes(*hbig, 2), stream, dbig, 0, nworld, 0,
                       1, integrate, mask);
    return hipGetLastError();
  }
  const StepFn fA = step_fn(host, 0), fB = step_fn(host, 1), fC = step_fn(host, 2);
  const StepFn fBL = newton_lat() ? step_fn(host, 3) : fB;
  const int nc = host.nrowclass;
  if (nc > 0 && !side) return hipErrorInvalidValue;
  const bool ovf = hbig && side && host.ovf_resolve;
  // Batch split: the worlds in nsplit contiguous ranges, each range's A -> B -> C chain on
  // its own stream.  The ranges are independent, so one range's launches fill the tail of
  // the other's (the last, partly filled round of workgroups per CU) and the launch gaps.
  // Measured: Go1 8192 worlds 4.91 -> 5.61 M env-steps/s at 2 splits (3: 5.47, 4: 5.38).
  // With row classes: launch_split_classes (flat fork / join); the default for those models
  // is one split (capi.cpp).  Masked forwards (reset worlds) stay one launch set.
  const int nsplit = (!mask && side) ? std::max(1, std::min(side->nsplit, kMaxSplit)) : 1;
  static const bool pipe = [] {
    const char* e = getenv("MJX355_CLASS_PIPE");
    return !e || atoi(e) != 0;
  }();

  if (nsplit > 1 && nc > 0) {
    // (diagnostic topology; the overflow re-solve is not wired into it)
    if (ovf) return hipErrorNotSupported;
    return launch_split_classes(host, dev, nworld, nsubstep, integrate, stream, side, nsplit, pipe);
  }
  hipStream_t sst[kMaxSplit];
  int wb[kMaxSplit + 1];
  for (int k = 0; k <= nsplit; k++) wb[k] = (int)(((long long)nworld * k) / nsplit);
  sst[0] = stream;
  hipError_t e = hipSuccess;
  if (nsplit > 1) {
    e = hipEventRecord(side->split_fork, stream);
    for (int k = 1; k < nsplit && e == hipSuccess; k++) {
      sst[k] = side->split[k];
      e = hipStreamWaitEvent(sst[k], side->split_fork, 0);
    }
    if (e != hipSuccess) return e;
  }
  // Row-class pipelines (nc > 0, one split): each class's Newton launch is followed on the
  // same stream by its phase C and then by the next substep's phase A for the same worlds,
  // so the bulk class's C and next A overlap the heavy class's Newton tail; the streams
  // join before the next classify.  MJX355_CLASS_PIPE=0: phase C / A over every world
  // after the join (diagnostic).
  // Models without row classes (Go1): each range's B -> C -> next substep's A as one launch
  // (step_chain over every world of the range), as the class pipelines do for a class, when
  // range_chain_default chose it.  Worlds listed for the re-solve skip the chain's B, C and
  // A; the re-solve chain then runs their next A too.  MJX355_RANGE_CHAIN=0/1 forces (A/B).
  static const int range_chain_env = [] {
    const char* e = getenv("MJX355_RANGE_CHAIN");
    return e ? atoi(e) : -1;
  }();
  const bool rchain = range_chain_env >= 0 ? range_chain_env != 0 : (side && side->range_chain);
  const StepFn fR = nc == 0 && !mask && rchain ? step_fn(host, 6) : nullptr;
  for (int sub = 0; sub < nsubstep; sub++) {
    const int last = sub == nsubstep - 1;
    const int apar = (sub & 1) ? kSelAPar : 0;  // phase A of this substep lists into parity sub & 1
    for (int k = 0; k < nsplit; k++) {
      const int w0 = wb[k], w1 = wb[k + 1], n = w1 - w0;
      if (n <= 0) continue;
      hipStream_t st = sst[k];
      const bool piped = nc > 0 && !mask && pipe;
      const bool nexta = piped || fR;  // the next substep's phase A runs behind this one's C
      if (!nexta || sub == 0)
        hipLaunchKernelGGL(fA, dim3(n), dim3(kWave), lds_bytes(host, 0), st, dev, w0, w1, k | apar,
                           last, integrate, mask);
      // the re-solve chain: forked after this substep's phase A (and classify), joined at the
      // end of the substep -- the empty chain overlaps the class launches
      // split batches: in line behind phase C on the split stream (a fork from a split
      // stream is a second-level fork, which breaks graph capture; capi.cpp).  Also in line
      // behind a range chain on an unsplit batch: the chain's B, C and fused next A skip the
      // listed worlds by ovf_flag[w], which the re-solve chain's next phase A rewrites, so a
      // concurrent re-solve could clear a flag before the range chain's workgroup for that
      // world reads it and the world would run one extra B -> C -> A.
      const bool ovf_inline = ovf && (nsplit > 1 || fR != nullptr);
      // (record the fork before the stream's next launch; launch the chain after it while
      // capturing: main_first)
      auto ovf_record = [&]() {
        if (!ovf || ovf_inline) return hipSuccess;
        return hipEventRecord(side->ovf_fork[k], st);
      };
      auto ovf_launch = [&]() {
        if (!ovf || ovf_inline) return hipSuccess;
        hipError_t e2 = hipStreamWaitEvent(side->ovf[k], side->ovf_fork[k], 0);
        if (e2 == hipSuccess)
          ovf_chain(host, dev, *hbig, dbig, side->ovf[k], k, w0, w1, sub, nsubstep, integrate,
                    nexta, false);
        return e2;
      };
      auto fork_ovf = [&]() {
        hipError_t e2 = ovf_record();
        return e2 == hipSuccess ? ovf_launch() : e2;
      };
      const bool mfirst = main_first(st);
      auto join_ovf = [&]() {
        if (!ovf) return hipSuccess;
        if (ovf_inline) {
          ovf_chain(host, dev, *hbig, dbig, st, k, w0, w1, sub, nsubstep, integrate, fR != nullptr, true);
          return hipSuccess;
        }
        hipError_t e2 = hipEventRecord(side->ovf_join[k], side->ovf[k]);
        if (e2 == hipSuccess) e2 = hipStreamWaitEvent(st, side->ovf_join[k], 0);
        return e2;
      };
      if (nc > 0 && mask) {
        // masked forward (a few reset worlds): one Newton launch at full capacity over the
        // masked worlds -- no classify launch, no fork/join latency on this short critical path
        // The grid is the whole batch and nearly every workgroup exits at once, so the launch
        // costs its dispatch rounds: with J read from the B pack in global memory (carve kLdsJG,
        // ~8 KB instead of the full fast carve's 31.8 KB) 16 workgroups fit a CU instead of 4.
        // MJX355_MASKED_JG=0: J in LDS (A/B)
        static const bool masked_jg = [] {
          const char* e = getenv("MJX355_MASKED_JG");
          return !e || atoi(e) != 0;
        }();
        const StepFn fMJ = masked_jg && newton_lat() ? step_fn(host, 9) : nullptr;
        hipLaunchKernelGGL(fMJ ? fMJ : fBL, dim3(n), dim3(kWave), lds_bytes(host, fMJ ? kLdsJG : 1), st,
                           dev, w0, w1, k, last, -1, mask);
        // (MJX355_MASKED_BIG=0) masked worlds past the fast carve: re-solved in line
        if (ovf) ovf_chain(host, dev, *hbig, dbig, st, k, w0, w1, sub, nsubstep, integrate, false, true);
      } else if (nc > 0) {
        hipLaunchKernelGGL(classify_kernel, dim3(1), dim3(kClassifyThreads), 0, st, dev, w0, w1,
                           k, mask);
        // MJX355_OVF_STREAM=1 (diagnostic, scripts/capture_probe*): the re-solve chain on a
        // stream of its own, forked here and joined after the class joins -- round 4's
        // topology, kept to reproduce its graph-replay crash
        if (ovf_stream_env() && (e = fork_ovf()) != hipSuccess) return e;
        // Newton by row class, concurrently: the full-capacity class (few worlds, long
        // per-world latency) first on a side stream so its blocks dispatch first, the middle
        // classes on further side streams, the smallest (most worlds) on the launch stream.
        // Measured: forking the side classes after the smallest makes the full class the tail
        // (B span 240 -> 255 us, G1).
        e = hipEventRecord(side->fork[k], st);
        if (e != hipSuccess) return e;
        // class c's stream: B, then (piped) C and the next substep's A of the same worlds --
        // as one launch (step_chain) unless MJX355_CHAIN=0
        auto class_chain = [&](hipStream_t cs, int cls) {
          const bool cjg = cls == 0 && newton_lat() && jg_mode(nworld) == 1;
          const StepFn fX = piped && chain_env(cls, nworld)
                                ? step_fn(host, cls == 0 && newton_lat() ? (cjg ? 11 : 7) : 6)
                                : nullptr;
          if (fX) {
            const int selx = k | (cls + 1) << 8 | (last ? 0 : kSelChainA) |
                             (((sub + 1) & 1) ? kSelAPar : 0) |
                             (sub + 1 == nsubstep - 1 ? kSelNextLast : 0);
            hipLaunchKernelGGL(fX, dim3(n), dim3(kWave), lds_chain(host, cls, !last, cjg), cs, dev,
                               w0, w1, selx, last, integrate, mask);
            return;
          }
          const int jg = cls == 0 ? jg_mode(nworld) : 0;
          const StepFn fJ = jg == 1 && newton_lat() ? step_fn(host, 9) : jg == 2 ? step_fn(host, 10) : nullptr;
          const StepFn fBH = cls == 0 && !fJ && heavy_cap(host) && newton_lat() ? step_fn(host, 12) : fBL;
          const int pr = fBH != fBL ? kSelPrio : 0;
          hipLaunchKernelGGL(cls ? fB : fJ ? fJ : fBH, dim3(n), dim3(kWave),
                             lds_bytes(host, cls ? 2 + cls : fJ ? kLdsJG : 1), cs, dev, w0, w1, k | pr, last,
                             cls, mask);
          if (!piped) return;
          hipLaunchKernelGGL(fC, dim3(n), dim3(kWave), lds_bytes(host, 2), cs, dev, w0, w1,
                             k | (cls + 1) << 8 | pr, last, integrate, mask);
          if (!last)
            hipLaunchKernelGGL(fA, dim3(n), dim3(kWave), lds_bytes(host, 0), cs, dev, w0, w1,
                               k | (cls + 1) << 8 | (((sub + 1) & 1) ? kSelAPar : 0) | pr,
                               sub + 1 == nsubstep - 1, integrate, mask);
        };
        for (int c = 0; c < nc; c++) {
          const int cls = c == 0 ? 0 : nc + 1 - c;  // 0, then nc, nc-1, ..., 2
          e = hipStreamWaitEvent(side->stream[k][c], side->fork[k], 0);
          if (e != hipSuccess) return e;
          class_chain(side->stream[k][c], cls);
          // the re-solve chain behind the full-capacity class (its stream ends well before the
          // bulk class's), not on a stream of its own: a further concurrent branch crashed
          // graph replay under torch's HIP runtime (two middle classes + the re-solve stream).
          // Measured ahead of that class instead: G1 -3 % (its 64 KiB workgroups then take
          // LDS from the bulk class's first Newton waves)
          if (c == 0 && ovf && !ovf_stream_env())
            ovf_chain(host, dev, *hbig, dbig, side->stream[k][0], k, w0, w1, sub, nsubstep,
                      integrate, piped, false);
        }
        class_chain(st, 1);
        for (int c = 0; c < nc; c++) {
          e = hipEventRecord(side->join[k][c], side->stream[k][c]);
          if (e == hipSuccess) e = hipStreamWaitEvent(st, side->join[k][c], 0);
          if (e != hipSuccess) return e;
        }
        if (ovf_stream_env() && (e = join_ovf()) != hipSuccess) return e;
        if (piped) continue;
      } else if (fR) {
        if ((e = ovf_record()) != hipSuccess) return e;
        if (!mfirst && (e = ovf_launch()) != hipSuccess) return e;
        const int selx = k | (last ? 0 : kSelChainA) | (((sub + 1) & 1) ? kSelAPar : 0) |
                         (sub + 1 == nsubstep - 1 ? kSelNextLast : 0);
        hipLaunchKernelGGL(fR, dim3(n), dim3(kWave), lds_chain(host, 0, !last), st, dev, w0, w1, selx,
                           last, integrate, mask);
        if (mfirst && (e = ovf_launch()) != hipSuccess) return e;
        if ((e = join_ovf()) != hipSuccess) return e;
        continue;
      } else {
        if ((e = ovf_record()) != hipSuccess) return e;
        if (!mfirst && (e = ovf_launch()) != hipSuccess) return e;
        // (MJX355_NEWTON_JG=2 on a model without row classes: J from global memory as well)
        const StepFn fBJ = newton_jg() == 2 ? step_fn(host, 10) : nullptr;  // (A/B only)
        hipLaunchKernelGGL(fBJ ? fBJ : fB, dim3(n), dim3(kWave), lds_bytes(host, fBJ ? kLdsJG : 1), st,
                           dev, w0, w1, k, last, 0, mask);
        if (mfirst && (e = ovf_launch()) != hipSuccess) return e;
      }
      hipLaunchKernelGGL(fC, dim3(n), dim3(kWave), lds_bytes(host, 2), st, dev, w0, w1, k, last,
                         integrate, mask);
      if (nc == 0 && (e = join_ovf()) != hipSuccess) return e;
    }
  }
  for (int k = 1; k < nsplit; k++) {
    e = hipEventRecord(side->split_join[k], sst[k]);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, side->split_join[k], 0);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// One-wave workgroups resident per CU at `bytes` of dynamic LDS, as measured on MI355X
// (scripts/lds_occupancy.hip: the first-round workgroups of a grid of spinning waves).  The
// hardware fits fewer than 160 KiB / bytes: 13,184 B hold 11 per CU, not 12 (12 need
// <= 12,800 B), 14,560 B 10, not 11 (11 need <= 14,080 B), 16,384 B 9, 8,192 B 18.
int lds_residency(size_t bytes) {
  static const struct { size_t max_bytes; int per_cu; } kTable[] = {
      {8192, 18}, {10240, 16}, {11264, 14}, {12800, 12}, {14080, 11}, {15360, 10}, {16384, 9},
      {20480, 8}, {32768, 4}};
  for (const auto& t : kTable)
    if (bytes <= t.max_bytes) return t.per_cu;
  return bytes > 0 ? std::max(1, (int)((size_t)147456 / bytes)) : 32;
}

// The range chain runs phases A and C at the Newton kernel's residency (registers and the
// largest carve).  Measured (Go1, 24 / 96 carve, two ranges, two interleaved rounds on one
// box): flat 4,096 worlds (2,048 per range) 5.25 -> 5.60 M env-steps/s, rough 8,192 (4,096
// per range) 4.57 -> 4.82 M, flat 8,192 7.38 -> 7.07 M.  A range that fits one residency
// round of the chain gains (two launch ramps and gaps per substep go); so does a model with
// terrain collision, whose long per-world phase-A tails the chain's per-world flow absorbs;
// a flat range needing a second round loses the cheap phases' residency.
bool range_chain_default(const Params& host, int nworld, int nsplit) {
  const StepFn f = step_fn(host, 6);
  hipFuncAttributes fa;
  if (!f || hipFuncGetAttributes(&fa, (const void*)f) != hipSuccess) return false;
  const int regs = (fa.numRegs + 7) & ~7;
  const int per_cu = std::min(4 * (regs > 0 ? std::min(8, 512 / regs) : 8),
                              lds_residency(lds_chain(host, 0, true)));
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  const int per_range = (nworld + std::max(nsplit, 1) - 1) / std::max(nsplit, 1);
  return per_range <= per_cu * ncu || host.d.nstatic > 0;
}

int choose_row_classes(const Dims& d, int spec, int (&caps)[kRowClasses]) {
  for (int k = 0; k < kRowClasses; k++) caps[k] = 0;
  int n = 0;
  if (const char* e = getenv("MJX355_ROW_CLASSES")) {  // diagnostic: "44,80" or "" (none)
    for (const char* c = e; *c && n < kRowClasses;) {
      const int v = atoi(c);
      if (v > 0 && v < d.njmax && (n == 0 || v > caps[n - 1])) caps[n++] = v;
      while (*c && *c != ',') c++;
      if (*c == ',') c++;
    }
    return n;
  }
  hipFuncAttributes fa;
  Params hp{};
  hp.d = d;
  hp.spec = spec;
  if (hipFuncGetAttributes(&fa, (const void*)step_fn(hp, 1)) != hipSuccess) return 0;
  // wave64 on gfx950: 512 VGPRs per SIMD lane (granule 8), 4 SIMDs per CU
  const int regs = (fa.numRegs + 7) & ~7;
  const int top = 4 * (regs > 0 ? std::min(8, 512 / regs) : 8);  // register-bound worlds/CU
  // largest row capacity (multiple of 4) whose phase-B carve lets `w` worlds share a CU
  auto cap_for = [&](int w) {
    Dims ds = d;
    for (int r = (d.njmax - 1) & ~3; r >= 8; r -= 4) {
      ds.njmax = r;
      if (lds_residency((size_t)make_lds(ds, 1).total * 4) >= w) return r;
    }
    return 0;
  };
  if (lds_residency((size_t)make_lds(d, 1).total * 4) >= top) return 0;  // no need
  // One class below the register-bound residency, the rest at full capacity (gated at 5/6 of
  // it).  Measured with the round-3 full-form Hessian (G1 4096, B span per substep): one class
  // at 44 / 52 / 60 / 64 / 72 / 84 rows 202 / 196 / 197 / 197 / 203 / 198 us; two classes
  // (44+84, 44+64, 60+100) 207-216 us -- concurrent class launches crowd each other out
  // A class that at most doubles the full carve's residency does not repay the classify
  // launch and the fork/join (Go1 8192: full carve 8 worlds/CU, B + gaps 136 -> 153 us)
  // Since the Newton Hessian is staged in LTR form (round 4: 60 rows 4052 -> 3476 words) the
  // class sits at 11/12 of the register-bound residency (G1: 64 rows, 11 worlds/CU).  G1
  // env-steps/s, caps default-5/6 (72 rows, 10/CU) / 56 (12/CU) / 64 (11/CU): velocity 4096
  // 2.636 / 2.662 / 2.657 M, jump flat 16384 7.80 / 7.80 / 7.88 M, jump hfield 16384 4.81 /
  // 4.88 / 4.87 M, rough 4096 2.45 / 2.46 / 2.47 M, tracking 2.46 / 2.47 / 2.46 M.
  const int full_per_cu = lds_residency((size_t)make_lds(d, 1).total * 4);
  for (int w : {(5 * top) / 6}) {
    if (w < 8 || 2 * full_per_cu > w) continue;
    const int r = cap_for((11 * top) / 12);
    if (r > 0 && (n == 0 || r > caps[n - 1]) && n < kRowClasses) caps[n++] = r;
  }
  return n;
}

// Profiling marker: an empty one-wave kernel whose dispatches bracket a region of interest
// in a kernel trace (mjx_marker; the argument is the tag, visible in the trace only by order).
__global__ void marker_kernel(int tag) {
  (void)tag;
}

hipError_t launch_marker(int tag, hipStream_t stream) {
  hipLaunchKernelGGL(marker_kernel, dim3(1), dim3(kWave), 0, stream, tag);
  return hipGetLastError();
}

hipError_t launch_reset(const Dims& d, const DModel& m, const DData& dd, const uint8_t* mask,
                        int nworld, int con_stride, hipStream_t stream) {
  if (nworld <= 0) return hipSuccess;
  hipLaunchKernelGGL(reset_kernel, dim3(nworld), dim3(kWave), 0, stream, d, m, dd, mask, nworld,
                     con_stride);
  return hipGetLastError();
}

}  // namespace mjx

