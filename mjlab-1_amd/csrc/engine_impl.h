#pragma once
// engine_impl.h — the step kernels of the batched mj_step for MI355X (gfx950): one
// wavefront (64 lanes) per world.  Included by engine.hip (generic kernels) and by
// spec.hip (one translation unit per model specialisation of specs.inc).
//
// Each workgroup is ONE wave that owns ONE world.  The world's state and every
// intermediate (body frames, com-based inertias, mass matrix, contacts, dense
// constraint Jacobian, Newton Hessian) lives in that workgroup's LDS for the whole
// step, so HBM sees only the coalesced load of the state at the start and the
// coalesced store of state + API-visible kinematics at the end (the "algorithmic
// bytes" of DESIGN.md section 4).  Stages map to lanes as:
//   tree recursions  -> one lane per body of the current tree level (level-synchronous)
//   dof stages       -> one lane per dof (M rows, Jacobian columns, J^T f)
//   broad+narrowphase-> one lane per candidate geom pair, LDS-atomic append, then a
//                       64-lane bitonic sort on (pair, sub-contact) so contact order is
//                       deterministic and equals the CPU oracle's pair order
//   constraint rows  -> one lane per row
//   Cholesky / H     -> one lane per lower-triangle element (right-looking, in LDS)
// Semantics follow the reference's mujoco_warp.step (src/mjlab/sim/sim.py:267-273)
// stage by stage, restated in oracle/oracle.c (the parity checker).
#include <float.h>
#include <stdlib.h>
#include <algorithm>
#include <initializer_list>
#include <utility>
#include <math.h>

#include "engine.h"

// FMA contraction only within one expression (the front end's fmuladd), never across
// statements in the back end: one source line then rounds the same in every kernel it is
// inlined into (step_phase, the re-solve's step_ovf), so a world's substep is bit
// for bit the same whichever launch set ran it.
#pragma clang fp contract(on)

namespace mjx {

#define MINVAL 1e-15f
#define MINMU 1e-5f
#define MINIMP 0.0001f
#define MAXIMP 0.9999f


// --------------------------------------------------------------------------- device math
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 v3(const float* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ void st3(float* p, V3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float norm(V3 a) { return sqrtf(dot(a, a)); }
// row-major 3x3
__device__ __forceinline__ V3 mulv(const float* M, V3 v) {
  return {M[0] * v.x + M[1] * v.y + M[2] * v.z, M[3] * v.x + M[4] * v.y + M[5] * v.z,
          M[6] * v.x + M[7] * v.y + M[8] * v.z};
}
__device__ __forceinline__ V3 mulTv(const float* M, V3 v) {
  return {M[0] * v.x + M[3] * v.y + M[6] * v.z, M[1] * v.x + M[4] * v.y + M[7] * v.z,
          M[2] * v.x + M[5] * v.y + M[8] * v.z};
}
__device__ __forceinline__ void mat3mul(float* R, const float* A, const float* B) {
  float t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) R[i] = t[i];
}
struct Q4 { float w, x, y, z; };
__device__ __forceinline__ Q4 q4(const float* p) { return {p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ void st4(float* p, Q4 q) { p[0] = q.w; p[1] = q.x; p[2] = q.y; p[3] = q.z; }
__device__ __forceinline__ Q4 qmul(Q4 a, Q4 b) {
  return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
          a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x, a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}
__device__ __forceinline__ Q4 qnorm(Q4 q) {
  float n = sqrtf(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  if (n < MINVAL) return {1, 0, 0, 0};
  float s = 1.0f / n;
  return {q.w * s, q.x * s, q.y * s, q.z * s};
}
__device__ __forceinline__ void qmat(float* M, Q4 q) {
  q = qnorm(q);
  float w = q.w, x = q.x, y = q.y, z = q.z;
  M[0] = 1 - 2 * (y * y + z * z); M[1] = 2 * (x * y - w * z); M[2] = 2 * (x * z + w * y);
  M[3] = 2 * (x * y + w * z); M[4] = 1 - 2 * (x * x + z * z); M[5] = 2 * (y * z - w * x);
  M[6] = 2 * (x * z - w * y); M[7] = 2 * (y * z + w * x); M[8] = 1 - 2 * (x * x + y * y);
}
// q v q* for a unit quaternion (18 FMAs, no normalisation)
__device__ __forceinline__ V3 qrot(Q4 q, V3 v) {
  const V3 u = {q.x, q.y, q.z};
  const V3 t = cross(u, v) * 2.f;
  return v + t * q.w + cross(u, t);
}
__device__ __forceinline__ Q4 qaxisangle(V3 a, float ang) {
  float s = sinf(0.5f * ang);
  return {cosf(0.5f * ang), a.x * s, a.y * s, a.z * s};
}
// spatial algebra, vectors [ang; lin]
__device__ __forceinline__ void cross_motion(float* r, const float* v, const float* s) {
  V3 w = v3(v), u = v3(v + 3), a = v3(s), b = v3(s + 3);
  st3(r, cross(w, a));
  st3(r + 3, cross(w, b) + cross(u, a));
}
__device__ __forceinline__ void cross_force(float* r, const float* v, const float* f) {
  V3 w = v3(v), u = v3(v + 3), a = v3(f), b = v3(f + 3);
  st3(r, cross(w, a) + cross(u, b));
  st3(r + 3, cross(w, b));
}
__device__ __forceinline__ void inert_mul(float* r, const float* I, const float* v) {
  V3 w = v3(v), u = v3(v + 3), h = v3(I + 6);
  float m = I[9];
  V3 t = {I[0] * w.x + I[3] * w.y + I[4] * w.z, I[3] * w.x + I[1] * w.y + I[5] * w.z,
          I[4] * w.x + I[5] * w.y + I[2] * w.z};
  st3(r, t + cross(h, u));
  st3(r + 3, u * m - cross(h, w));
}
__device__ __forceinline__ float dot6(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

// --------------------------------------------------------------------------- wave utils
// Full-wave float sum, result wave-uniform.  DPP within each 16-lane row (quad swaps,
// half-row and row mirrors), then the four row totals via v_readlane: no LDS crossbar
// round trips (a __shfl_xor chain costs six ds_swizzle latencies).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
}
// min / max over the wave (same DPP pattern as wave_sum; all lanes must be active)
__device__ __forceinline__ float wave_min(float v) {
  v = fminf(v, dpp<0xB1>(v));
  v = fminf(v, dpp<0x4E>(v));
  v = fminf(v, dpp<0x141>(v));
  v = fminf(v, dpp<0x140>(v));
  const auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
  return fminf(fminf(rl(0), rl(16)), fminf(rl(32), rl(48)));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  const auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
  return fmaxf(fmaxf(rl(0), rl(16)), fmaxf(rl(32), rl(48)));
}
__device__ __forceinline__ int wave_excl_scan(int v, int lane, int* total) {
  int x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  *total = __shfl(x, kWave - 1);
  return x - v;
}
// A workgroup is exactly one wavefront and LDS operations of a wavefront execute in
// issue order, so cross-lane LDS hand-offs need only a compiler barrier (no s_barrier,
// no lgkmcnt drain).  MJX_SYNCTHREADS=1 restores __syncthreads() for A/B checks.
#ifndef MJX_SYNCTHREADS
__device__ __forceinline__ void sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
#else
__device__ __forceinline__ void sync() { __syncthreads(); }
#endif

#define MF(f) (m.f + (size_t)w * m.f##_ws)

// Diagnostic build only (-DMJX_STAMPS): per-stage s_memtime deltas, accumulated in
// registers and added to D.prof once per wave at kernel end (STAMP_FLUSH) -- per-stamp global
// atomics sit in vmcnt and would charge their contention to the next memory wait.
#ifdef MJX_STAMPS
#define STAMP(k)                                                                 \
  do {                                                                           \
    __builtin_amdgcn_s_waitcnt(0xC07F);                                          \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
    stamp_acc[k] += t_ - stamp_prev;                                             \
    stamp_prev = t_;                                                             \
  } while (0)
// SUBSTAMP(k): nested split of the Newton stage into slots 16+ (does not advance STAMP).
#define SUBSTAMP(k)                                                              \
  do {                                                                           \
    __builtin_amdgcn_s_waitcnt(0xC07F);                                          \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                         \
    stamp_acc[16 + (k)] += t_ - sub_prev;                                        \
    sub_prev = t_;                                                               \
  } while (0)
// Only worlds with at least P->stamp_minrows constraint rows this substep are counted
// (MJX355_STAMP_MINROWS: the breakdown of the heavy worlds); slot 47 counts flushes.
#define STAMP_FLUSH()                                                            \
  do {                                                                           \
    if (lane == 0 && D.nefc[w] >= P->stamp_minrows) {                            \
      stamp_acc[47] = 1;                                                         \
      for (int k_ = 0; k_ < 48; k_++)                                            \
        if (stamp_acc[k_]) atomicAdd((unsigned long long*)&D.prof[k_], stamp_acc[k_]); \
    }                                                                            \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#define SUBSTAMP(k) do {} while (0)
#define STAMP_FLUSH() do {} while (0)
#endif

// --------------------------------------------------------------------------- tiled SPD algebra
// The nv x nv SPD systems (mass matrix, Newton Hessian, implicit-integration matrix) are
// padded to NVP = 4*ceil(nv/4) and split into 4x4 tiles of the lower triangle; lane l owns
// tiles l and l+64 (at most 2, so NVP <= 60).  Tiles live in registers through assembly
// and factorization; the Cholesky factor is published to LDS (row stride NVP) for the
// triangular solves.  Padding rows/cols are identity, so padded unknowns solve to 0.
struct Tiles {
  int nb, ntile;
  int bi[2], bj[2];
  bool own[2];
};
__device__ __forceinline__ Tiles make_tiles(int nvp, int lane) {
  Tiles t;
  t.nb = nvp >> 2;
  t.ntile = t.nb * (t.nb + 1) / 2;
#pragma unroll
  for (int s = 0; s < 2; s++) {
    int idx = lane + kWave * s;
    t.own[s] = idx < t.ntile;
    int bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= idx) bi++;
    t.bi[s] = bi;
    t.bj[s] = idx - bi * (bi + 1) / 2;
  }
  return t;
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4v(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ void tiles_load(float (&A)[2][16], const Tiles& T, const float* Mm, int nvp) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float4 v = ld4(Mm + (4 * T.bi[s] + r) * nvp + 4 * T.bj[s]);
      A[s][4 * r + 0] = v.x; A[s][4 * r + 1] = v.y; A[s][4 * r + 2] = v.z; A[s][4 * r + 3] = v.w;
    }
  }
}
// A += sum_k D[act[k]] * J[act[k], iblock]^T J[act[k], jblock]
__device__ __forceinline__ void tiles_add_jtdj(float (&A)[2][16], const Tiles& T, const float* J,
                                               const float* Dv, const int* act, int nact, int nvp) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
    const int oi = 4 * T.bi[s], oj = 4 * T.bj[s];
    int k = 0;
    for (; k + 1 < nact; k += 2) {
      int r0 = act[k], r1 = act[k + 1];
      float4 a0 = ld4(J + r0 * nvp + oi), b0 = ld4(J + r0 * nvp + oj);
      float4 a1 = ld4(J + r1 * nvp + oi), b1 = ld4(J + r1 * nvp + oj);
      float d0 = Dv[r0], d1 = Dv[r1];
      float ai0[4] = {a0.x, a0.y, a0.z, a0.w}, bj0[4] = {b0.x * d0, b0.y * d0, b0.z * d0, b0.w * d0};
      float ai1[4] = {a1.x, a1.y, a1.z, a1.w}, bj1[4] = {b1.x * d1, b1.y * d1, b1.z * d1, b1.w * d1};
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) A[s][4 * r + c] += ai0[r] * bj0[c] + ai1[r] * bj1[c];
    }
    if (k < nact) {
      int r0 = act[k];
      float4 a0 = ld4(J + r0 * nvp + oi), b0 = ld4(J + r0 * nvp + oj);
      float d0 = Dv[r0];
      float ai0[4] = {a0.x, a0.y, a0.z, a0.w}, bj0[4] = {b0.x * d0, b0.y * d0, b0.z * d0, b0.w * d0};
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) A[s][4 * r + c] += ai0[r] * bj0[c];
    }
  }
}
// The same sum on the matrix cores (built with -DMJX_JTDJ_MFMA=1; A/B against the VALU
// tiles above): v_mfma_f32_16x16x4_f32 (exact fp32, 32 cycles issue per SIMD) over 16x16
// blocks (I, J), I >= J, of the padded Hessian, 4 active rows per instruction.  Lane l
// supplies A[i = l & 15][k = l >> 4] = J[act[k0 + k], 16 I + i] and B[k][j = l & 15] =
// D * J[act[k0 + k], 16 J + j]; the accumulator holds block row (l >> 4) * 4 + reg, column
// l & 15 (cdna_hip_programming.md section 3).  Lm (row stride nvp) must already hold M; the
// blocks are added into it (lower triangle and the diagonal blocks).  Ends synced.
#ifndef MJX_JTDJ_MFMA
#define MJX_JTDJ_MFMA 0
#endif
typedef float mfma_f4 __attribute__((ext_vector_type(4)));
template <int NR>
__device__ __forceinline__ void mfma_add_jtdj(float* Lm, const float* J, const float* Dv,
                                              const int* act, int nact, int nvp, int lane) {
  // one block at a time (one 4-register accumulator live: the Newton kernel sits at the
  // 3-waves-per-SIMD register bound)
  constexpr int NB = (NR + 15) / 16;
  const int i16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int I = 0; I < NB; I++) {
#pragma unroll
    for (int Jb = 0; Jb <= I; Jb++) {
      mfma_f4 acc = {0.f, 0.f, 0.f, 0.f};
      const int ca = 16 * I + i16, cb = 16 * Jb + i16;
      for (int k0 = 0; k0 < nact; k0 += 4) {
        const int k = k0 + kq;
        const bool in = k < nact;
        const int r = in ? act[k] : 0;
        const float a = (in && ca < nvp) ? J[r * nvp + ca] : 0.f;
        const float bv = (in && cb < nvp) ? J[r * nvp + cb] * Dv[r] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int row = 16 * I + 4 * kq + q;
        if (row < nvp && cb < nvp) Lm[row * nvp + cb] += acc[q];
      }
    }
  }
  sync();
}
// out[i] = Mm[i,:] . v for i < nrow (row stride nvp), v broadcast-read as float4.
__device__ __forceinline__ void matvec_rows(float* out, const float* Mm, const float* v, int nrow,
                                            int nvp, int lane) {
  const int nb = nvp >> 2;
  for (int i = lane; i < nrow; i += kWave) {
    const float* row = Mm + i * nvp;
    float s0 = 0.f, s1 = 0.f;
    int k = 0;
    for (; k + 1 < nb; k += 2) {
      float4 a = ld4(row + 4 * k), b = ld4(v + 4 * k);
      float4 c = ld4(row + 4 * k + 4), e = ld4(v + 4 * k + 4);
      s0 += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
      s1 += c.x * e.x + c.y * e.y + c.z * e.z + c.w * e.w;
    }
    if (k < nb) {
      float4 a = ld4(row + 4 * k), b = ld4(v + 4 * k);
      s0 += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    }
    out[i] = s0 + s1;
  }
}
// out[c] = sum_k J[act[k], c] * wv[act[k]] (c < nvp).  Lanes split (column block, row
// group); partial sums reduced through `part` (>= 64*4 floats).  Ends with a sync.
__device__ __forceinline__ void jt_mul(float* out, const float* J, const float* wv, const int* act, int nact,
                       int nvp, int lane) {
  // lane = g * nb + cb: column block cb (4 columns) summed over the rows k = g (mod ng),
  // then the ng group partials are folded by a fixed shuffle tree (no LDS scratch, so the
  // Newton factor in the H slot survives across iterations)
  const int nb = nvp >> 2;
  const int ng = kWave / nb;
  const int cb = lane % nb, g = lane / nb;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g < ng) {
    for (int k = g; k < nact; k += ng) {
      int r = act[k];
      float4 j = ld4(J + r * nvp + 4 * cb);
      float wr = wv[r];
      acc.x += j.x * wr; acc.y += j.y * wr; acc.z += j.z * wr; acc.w += j.w * wr;
    }
  }
  for (int off = 1; off < ng; off <<= 1) {
    const int src = min(lane + off * nb, kWave - 1);
    const bool take = g + off < ng;
    const float x = __shfl(acc.x, src), y = __shfl(acc.y, src);
    const float z = __shfl(acc.z, src), w = __shfl(acc.w, src);
    if (take) { acc.x += x; acc.y += y; acc.z += z; acc.w += w; }
  }
  if (g == 0) st4v(out + 4 * cb, acc);
  sync();
}
// Compact the rows with jar < 0 into act[]; returns the count (wave-uniform).  sig holds
// the active set of the previous call as 64-row ballots; *same is set when it is unchanged
// (then H = M + J_act^T D J_act is unchanged too).  Sets over 4*64 rows never compare same.
__device__ __forceinline__ int build_active(int* act, const float* jar, int nefc, int lane,
                                            unsigned long long (&sig)[4], bool* same,
                                            int* nchg = nullptr) {
  int base = 0, chg = 0;
  bool eq = nefc <= 4 * kWave;
  for (int r0 = 0, k = 0; r0 < nefc; r0 += kWave, k++) {
    int r = r0 + lane;
    bool f = r < nefc && jar[r] < 0.f;
    unsigned long long bal = __ballot(f);
    if (f) act[base + __popcll(bal & ((1ull << lane) - 1ull))] = r;
    base += __popcll(bal);
    if (k < 4) {
      eq = eq && bal == sig[k];
      chg += __popcll(bal ^ sig[k]);
      sig[k] = bal;
    }
  }
  *same = eq;
  if (nchg) *nchg = chg;
  return base;
}

// build_active for nefc <= 64 with row `lane`'s jar in a register (lanes past nefc: 0)
__device__ __forceinline__ int build_active1(int* act, float rja, int nefc, int lane,
                                             unsigned long long (&sig)[4], bool* same,
                                             int* nchg = nullptr) {
  const bool f = lane < nefc && rja < 0.f;
  const unsigned long long bal = __ballot(f);
  if (f) act[__popcll(bal & ((1ull << lane) - 1ull))] = lane;
  *same = nefc <= 0 || bal == sig[0];
  if (nchg) *nchg = nefc > 0 ? __popcll(bal ^ sig[0]) : 0;
  if (nefc > 0) sig[0] = bal;
  return __popcll(bal);
}

// --------------------------------------------------------------------------- register-row SPD
// Lane i holds row i of an nvp x nvp SPD matrix in NR registers (NR = compile-time row
// length >= nvp; rows/cols >= nvp are identity).  Cholesky and both triangular solves run
// as v_readlane broadcast chains: no LDS round trips and no single-lane sections.
__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// The lane index as a value the compiler cannot hoist: the per-column lane tests of the
// register-row code (c < lane, c == lane) are then formed where they are used (one v_cmp
// + v_cndmask each) instead of being hoisted out of the Newton loop as ~36 SGPR-pair masks
// that spill into VGPR lanes and turn every select into an exec-mask branch.
__device__ __forceinline__ int opaque_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}
template <int NR>
__device__ __forceinline__ void rows_load(float (&A)[NR], const float* Mm, int nvp, int lane) {
  const int row = lane < nvp ? lane : 0;
#pragma unroll
  for (int c = 0; c < NR; c += 4) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nvp) v = ld4(Mm + row * nvp + c);
    A[c] = v.x; A[c + 1] = v.y; A[c + 2] = v.z; A[c + 3] = v.w;
  }
  if (NR > nvp || kWave > NR) {  // identity rows past nvp (wave-uniform test)
    const int ln = opaque_lane(lane);
    const bool pad = ln >= nvp;
#pragma unroll
    for (int c = 0; c < NR; c++) A[c] = pad ? (c == ln ? 1.f : 0.f) : A[c];
  }
}
// In-place blocked right-looking Cholesky of the lower triangle: afterwards A[c] (c <= lane)
// is L[lane][c] and rdiag = 1/L[lane][lane].  Entries above the diagonal are scratch; they
// never feed the lower part.  Columns go in blocks of 4: the diagonal block is factored with
// v_readlane broadcasts (6 per block), then each lane publishes its 4 block entries to
// `cb` (LDS, 4*64 floats: every lane writes, no branch) and every lane reads the block rows of the trailing columns back
// as broadcast float4s -- one LDS round trip per 4 columns instead of one v_readlane per
// trailing element (630 for NR 36).
// PIPE (the latency kernel): each trailing group's four broadcast reads are issued before the
// previous group's FMAs, so the LDS latency is paid once per block instead of once per group
// (16 more VGPRs; -10 % factor latency on one wave, scripts/chol_bench.hip).
template <int NR, bool PIPE = false>
__device__ __forceinline__ void rows_chol(float (&A)[NR], float& rdiag, float* cb, int nvp, int lane) {
  static_assert(NR % 4 == 0, "register rows come in column blocks of 4");
  rdiag = 1.f;
  // Padding rows/cols (>= nvp) are identity/zero, so the full NR sweep is exact there:
  // no per-step guards (guards get hoisted into spilled SGPR masks).
#pragma unroll
  for (int j0 = 0; j0 < NR; j0 += 4) {
    const int ln = opaque_lane(lane);
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = j0 + t;
      const float r = __builtin_amdgcn_rsqf(fmaxf(rl(A[j], j), MINVAL));
      A[j] *= r;
      rdiag = ln == j ? r : rdiag;
#pragma unroll
      for (int u = t + 1; u < 4; u++) A[j0 + u] = fmaf(-A[j], rl(A[j], j0 + u), A[j0 + u]);
    }
    if (j0 + 4 < NR) {
      st4v(cb + 4 * lane, make_float4(A[j0], A[j0 + 1], A[j0 + 2], A[j0 + 3]));  // all 64 lanes (no branch)
      sync();
      if constexpr (PIPE) {
        float4 c[4], n[4];
#pragma unroll
        for (int u = 0; u < 4; u++) c[u] = ld4(cb + 4 * (j0 + 4 + u));
#pragma unroll
        for (int k0 = j0 + 4; k0 < NR; k0 += 4) {
          if (k0 + 4 < NR) {
#pragma unroll
            for (int u = 0; u < 4; u++) n[u] = ld4(cb + 4 * (k0 + 4 + u));
          }
          float q[4];
#pragma unroll
          for (int u = 0; u < 4; u++) q[u] = fmaf(-A[j0], c[u].x, A[k0 + u]);
#pragma unroll
          for (int u = 0; u < 4; u++) q[u] = fmaf(-A[j0 + 1], c[u].y, q[u]);
#pragma unroll
          for (int u = 0; u < 4; u++) q[u] = fmaf(-A[j0 + 2], c[u].z, q[u]);
#pragma unroll
          for (int u = 0; u < 4; u++) A[k0 + u] = fmaf(-A[j0 + 3], c[u].w, q[u]);
#pragma unroll
          for (int u = 0; u < 4; u++) c[u] = n[u];
        }
        sync();
        continue;
      }
      // trailing columns in groups of 4 (at most 16 broadcast VGPRs in flight: unbounded,
      // the scheduler hoists every read of the block and the kernel loses occupancy)
#pragma unroll
      for (int k0 = j0 + 4; k0 < NR; k0 += 4) {
        float4 c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) c[u] = ld4(cb + 4 * (k0 + u));  // row k of the block: broadcast
#pragma unroll
        for (int u = 0; u < 4; u++)
          A[k0 + u] = fmaf(-A[j0 + 3], c[u].w, fmaf(-A[j0 + 2], c[u].z,
                      fmaf(-A[j0 + 1], c[u].y, fmaf(-A[j0], c[u].x, A[k0 + u]))));
      }
      sync();  // the next block's publish follows these reads
    }
  }
  (void)nvp;
}
// The triangular solves run on scaled copies of L so that each of their 2*NR sequential
// steps is one v_readlane plus one FMA (no per-step rescale or select):
//   forward  L y = b   as u = diag(L) y:  u_j = b_j - sum_{k<j} M_jk u_k,  M_jk = L_jk / L_kk
//   backward L^T x = y as v = diag(L) x:  v_j = y_j - sum_{k>j} N_kj v_k,  N_kj = L_kj / L_kk
// M is column-scaled (register rows, rows_fwd_rows), N row-scaled (published to LDS by
// rows_store_strict and read back by columns).
// Publish N (row stride nvp): strictly-lower part, 1/L[i][i] on the diagonal, zeros above.
template <int NR>
__device__ __forceinline__ void rows_store_strict(const float (&A)[NR], float rd, float* Lm, int nvp,
                                                  int lane) {
  if (lane >= nvp) return;
  const int ln = opaque_lane(lane);
#pragma unroll
  for (int c = 0; c < NR; c += 4)
    if (c < nvp)
      st4v(Lm + lane * nvp + c,
           make_float4(c < ln ? A[c] * rd : c == ln ? rd : 0.f,
                       c + 1 < ln ? A[c + 1] * rd : c + 1 == ln ? rd : 0.f,
                       c + 2 < ln ? A[c + 2] * rd : c + 2 == ln ? rd : 0.f,
                       c + 3 < ln ? A[c + 3] * rd : c + 3 == ln ? rd : 0.f));
}
// Factor rows L (rows_chol) -> forward rows M (strictly lower, column-scaled).
template <int NR>
__device__ __forceinline__ void rows_fwd_rows(float (&A)[NR], float rd, int lane) {
  const int ln = opaque_lane(lane);
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const float s = rl(rd, k);  // outside the select: a readlane under a lane test is a branch
    A[k] = k < ln ? A[k] * s : 0.f;
  }
}
// Forward rows M of a factor published by rows_store_strict (M_jk = N_jk L_jj / L_kk), and
// this lane's 1/L[i][i].
template <int NR>
__device__ __forceinline__ void rows_load_factor(float (&A)[NR], float& rd, const float* Lm, int nvp,
                                                 int lane) {
  rows_load<NR>(A, Lm, nvp, lane);
  const int ln = opaque_lane(lane);
  const int dl = ln < nvp ? ln : 0;
  const float dv = Lm[dl * nvp + dl];  // unconditional load, then select (no exec branch)
  rd = ln < nvp ? dv : 1.f;
  const float ljj = __builtin_amdgcn_rcpf(rd);
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const float s = rl(rd, k);
    A[k] = k < ln ? A[k] * (s * ljj) : 0.f;
  }
}
// x (lane i holds x[i]) <- (L L^T)^-1 x, from the forward rows M (registers) and the columns
// of N in Lm (rows_store_strict, then synced).  Lanes >= nvp hold x = 0 and stay 0.
template <int NR>
__device__ __forceinline__ float rows_solve(const float (&M)[NR], float rdiag, const float* Lm,
                                            float x, int nvp, int lane) {
  float u = x;
#pragma unroll
  for (int j = 0; j < NR; j++) u = fmaf(-M[j], rl(u, j), u);  // M[j] = 0 on lanes <= j
  float Nc[NR];
  const int ln = opaque_lane(lane);
  const int col = ln < nvp ? ln : 0;
#pragma unroll
  for (int j = 0; j < NR; j++) {
    const float t = Lm[(j < nvp ? j : 0) * nvp + col];  // load, then select (no exec branch)
    Nc[j] = (j < nvp && j > ln) ? t : 0.f;
  }
  float v = u * rdiag;  // y = u / L_jj: the backward sweep starts at v = y
#pragma unroll
  for (int j = NR - 1; j >= 0; j--) v = fmaf(-Nc[j], rl(v, j), v);
  return v * rdiag;
}
// The same three steps on a factor kept in lower-tile-rows form (LTR, carve.h: row i holds
// columns [0, 4(i/4 + 1)) at ltr_off(i)): the phase A -> C hand-off of the implicit factor,
// 720 instead of 1296 floats for nvp 36.  Columns past a row's tiles are zero in the full
// form (rows_store_strict), so nothing else changes.
template <int NR>
__device__ __forceinline__ void rows_store_strict_ltr(const float (&A)[NR], float rd, float* Lp, int nvp,
                                                      int lane) {
  if (lane >= nvp) return;
  const int ln = opaque_lane(lane);
  float* row = Lp + ltr_off(lane);
  const int len = 4 * ((lane >> 2) + 1);
#pragma unroll
  for (int c = 0; c < NR; c += 4)
    if (c < len)
      st4v(row + c, make_float4(c < ln ? A[c] * rd : c == ln ? rd : 0.f,
                                c + 1 < ln ? A[c + 1] * rd : c + 1 == ln ? rd : 0.f,
                                c + 2 < ln ? A[c + 2] * rd : c + 2 == ln ? rd : 0.f,
                                c + 3 < ln ? A[c + 3] * rd : c + 3 == ln ? rd : 0.f));
}
// Row `row` of an LTR matrix as a full register row WITHOUT masking: columns past the row's
// tiles hold the next rows' entries (every read stays inside the ltr_size(nvp) array: the
// last block's rows are full).  For the callers whose entries above the diagonal are scratch
// or dropped by their own k < lane select; one base address and immediate offsets, where a
// per-lane row length costs a select per column (+18 VGPRs in the Newton kernel).
template <int NR>
__device__ __forceinline__ void rows_load_ltr_span(float (&A)[NR], const float* rp, int nvp) {
#pragma unroll
  for (int c = 0; c < NR; c += 4) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nvp) v = ld4(rp + c);
    A[c] = v.x; A[c + 1] = v.y; A[c + 2] = v.z; A[c + 3] = v.w;
  }
}
template <int NR>
__device__ __forceinline__ void rows_load_factor_ltr(float (&A)[NR], float& rd, const float* Lp,
                                                     int nvp, int lane) {
  const int ln = opaque_lane(lane);
  const int row = ln < nvp ? ln : 0;
  const float* rp = Lp + ltr_off(row);
  rows_load_ltr_span<NR>(A, rp, nvp);  // entries k >= lane are zeroed below
  const float dv = rp[row];
  rd = ln < nvp ? dv : 1.f;
  const float ljj = __builtin_amdgcn_rcpf(rd);
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const float s = rl(rd, k);
    A[k] = k < ln ? A[k] * (s * ljj) : 0.f;
  }
}
// rows_load_factor_ltr in two halves: the loads (issued early -- phase C puts them in flight
// with its pack's LDS-DMA, so the factor's latency overlaps the pack's) and the scaling.
template <int NR>
__device__ __forceinline__ void rows_load_factor_ltr_raw(float (&A)[NR], float& dv, const float* Lp,
                                                         int nvp, int lane) {
  const int ln = opaque_lane(lane);
  const int row = ln < nvp ? ln : 0;
  const float* rp = Lp + ltr_off(row);
  const int len = 4 * ((row >> 2) + 1);
#pragma unroll
  for (int c = 0; c < NR; c += 4) {
    const float4 v = ld4(rp + (c < len ? c : 0));
    const bool in = c < len;
    A[c] = in ? v.x : 0.f; A[c + 1] = in ? v.y : 0.f; A[c + 2] = in ? v.z : 0.f; A[c + 3] = in ? v.w : 0.f;
  }
  dv = rp[row];
}
// Register rows of a matrix in LTR form (the lower tiles, unmasked), identity rows past nvp:
// rows_load's counterpart for the blocked Cholesky, whose entries above the diagonal are
// scratch.
template <int NR>
__device__ __forceinline__ void rows_load_ltr(float (&A)[NR], const float* Lp, int nvp, int lane) {
  rows_load_ltr_span<NR>(A, Lp + ltr_off(lane < nvp ? lane : 0), nvp);
  if (NR > nvp || kWave > NR) {
    const int ln = opaque_lane(lane);
    const bool pad = ln >= nvp;
#pragma unroll
    for (int c = 0; c < NR; c++) A[c] = pad ? (c == ln ? 1.f : 0.f) : A[c];
  }
}
template <int NR>
__device__ __forceinline__ void rows_scale_factor_ltr(float (&A)[NR], float& rd, float dv, int nvp,
                                                      int lane) {
  const int ln = opaque_lane(lane);
  rd = ln < nvp ? dv : 1.f;
  const float ljj = __builtin_amdgcn_rcpf(rd);
#pragma unroll
  for (int k = 0; k < NR; k++) {
    const float s = rl(rd, k);
    A[k] = k < ln ? A[k] * (s * ljj) : 0.f;
  }
}
template <int NR>
__device__ __forceinline__ float rows_solve_ltr(const float (&M)[NR], float rdiag, const float* Lp,
                                                float x, int nvp, int lane) {
  float u = x;
#pragma unroll
  for (int j = 0; j < NR; j++) u = fmaf(-M[j], rl(u, j), u);
  float Nc[NR];
  const int ln = opaque_lane(lane);
  const int col = ln < nvp ? ln : 0;
#pragma unroll
  for (int j = 0; j < NR; j++) {
    const float t = Lp[ltr_off(j < nvp ? j : 0) + col];  // inside the LTR block, then select
    Nc[j] = (j < nvp && j > ln) ? t : 0.f;
  }
  float v = u * rdiag;
#pragma unroll
  for (int j = NR - 1; j >= 0; j--) v = fmaf(-Nc[j], rl(v, j), v);
  return v * rdiag;
}
// LDS matrix (row stride nvp) -> its lower 4x4 tiles in LTR form (any memory), chunk k of 4
// floats at 4k: block b of 4 rows starts at chunk 2 b (b + 1), each row takes b + 1 chunks.
__device__ __forceinline__ void store_ltr(float* dst, const float* Mm, int nvp, int lane) {
  const int nchunk = ltr_size(nvp) >> 2;
  for (int k = lane; k < nchunk; k += kWave) {
    int b = 0;
    while (2 * (b + 1) * (b + 2) <= k) b++;
    const int kk = k - 2 * b * (b + 1), r = kk / (b + 1), cc = kk - r * (b + 1);
    st4v(dst + 4 * k, ld4(Mm + (4 * b + r) * nvp + 4 * cc));
  }
}
// Lower 4x4 tiles from a matrix in LTR form (tiles_load's layout counterpart).
__device__ __forceinline__ void tiles_load_ltr(float (&A)[2][16], const Tiles& T, const float* Mp) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float4 v = ld4(Mp + ltr_off(4 * T.bi[s] + r) + 4 * T.bj[s]);
      A[s][4 * r + 0] = v.x; A[s][4 * r + 1] = v.y; A[s][4 * r + 2] = v.z; A[s][4 * r + 3] = v.w;
    }
  }
}
// Tiles (lower 4x4 blocks) -> LDS matrix (row stride nvp), for rows_load.
__device__ __forceinline__ void tiles_store(const float (&A)[2][16], const Tiles& T, float* Mm, int nvp) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
#pragma unroll
    for (int r = 0; r < 4; r++)
      st4v(Mm + (4 * T.bi[s] + r) * nvp + 4 * T.bj[s],
           make_float4(A[s][4 * r], A[s][4 * r + 1], A[s][4 * r + 2], A[s][4 * r + 3]));
  }
}
// Tiles -> the full symmetric LDS matrix: the lower tiles and, off the diagonal, their
// transposes (rows_load_rev reads the natural upper triangle).
__device__ __forceinline__ void tiles_store_sym(const float (&A)[2][16], const Tiles& T, float* Mm,
                                                int nvp) {
  tiles_store(A, T, Mm, nvp);
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s] || T.bi[s] == T.bj[s]) continue;
#pragma unroll
    for (int c = 0; c < 4; c++)
      st4v(Mm + (4 * T.bj[s] + c) * nvp + 4 * T.bi[s],
           make_float4(A[s][c], A[s][4 + c], A[s][8 + c], A[s][12 + c]));
  }
}
// Phase B stages the Newton Hessian in LTR form (720 floats for nvp 36, not 1296: the
// bulk row class's LDS then admits 11 worlds per CU instead of 10).  Tiles -> LTR in the
// natural order, for rows_load_ltr.
__device__ __forceinline__ void tiles_store_ltr(const float (&A)[2][16], const Tiles& T, float* Lp) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
#pragma unroll
    for (int r = 0; r < 4; r++)
      st4v(Lp + ltr_off(4 * T.bi[s] + r) + 4 * T.bj[s],
           make_float4(A[s][4 * r], A[s][4 * r + 1], A[s][4 * r + 2], A[s][4 * r + 3]));
  }
}
// Tiles -> the REVERSED matrix (index p <-> nvp-1-p) in LTR form: tile (bi, bj) lands at
// reversed block (nb-1-bj, nb-1-bi), transposed off the diagonal, flipped on it.  The values
// are the ones tiles_store_sym + rows_load_rev read (the transposed copy above the diagonal,
// each diagonal tile's own entries), so the factor is bit for bit the full-layout one.
__device__ __forceinline__ void tiles_store_rev_ltr(const float (&A)[2][16], const Tiles& T, float* Lp) {
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
    const int I = T.nb - 1 - T.bj[s], J = T.nb - 1 - T.bi[s];
    const bool dg = T.bi[s] == T.bj[s];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float v[4];
#pragma unroll
      for (int c = 0; c < 4; c++) v[c] = dg ? A[s][4 * (3 - r) + 3 - c] : A[s][4 * (3 - c) + 3 - r];
      st4v(Lp + ltr_off(4 * I + r) + 4 * J, make_float4(v[0], v[1], v[2], v[3]));
    }
  }
}
// out = A v for the symmetric matrix held as lower 4x4 register tiles (diagonal blocks
// full); each tile contributes its block and, off the diagonal, its transpose, through LDS
// float atomics.  Ends synced.
__device__ __forceinline__ void tiles_symv(const float (&A)[2][16], const Tiles& T, const float* v,
                                           float* out, int nvp, int lane) {
  for (int i = lane; i < nvp; i += kWave) out[i] = 0.f;
  sync();
#pragma unroll
  for (int s = 0; s < 2; s++) {
    if (!T.own[s]) continue;
    const int bi = T.bi[s], bj = T.bj[s];
    const float4 vj = ld4(v + 4 * bj);
#pragma unroll
    for (int r = 0; r < 4; r++)
      atomicAdd(out + 4 * bi + r, A[s][4 * r] * vj.x + A[s][4 * r + 1] * vj.y +
                                      A[s][4 * r + 2] * vj.z + A[s][4 * r + 3] * vj.w);
    if (bi != bj) {
      const float4 vi = ld4(v + 4 * bi);
#pragma unroll
      for (int c = 0; c < 4; c++)
        atomicAdd(out + 4 * bj + c, A[s][c] * vi.x + A[s][4 + c] * vi.y + A[s][8 + c] * vi.z +
                                        A[s][12 + c] * vi.w);
    }
  }
  sync();
}
// Factor the nvp x nvp SPD matrix in Mm (row stride nvp) and solve for vector v (LDS,
// length nvp) in place.  Lm (nvp*nvp) receives the strictly-lower factor.  Lm may alias Mm.
template <int NR>
__device__ __forceinline__ void spd_factor_solve(const float* Mm, const float* diag_add, float* Lm,
                                                 float* v, float* cb, int nvp, int lane) {
  float A[NR];
  rows_load<NR>(A, Mm, nvp, lane);
  if (diag_add && lane < nvp) {
#pragma unroll
    for (int c = 0; c < NR; c++) A[c] += c == lane ? diag_add[lane] : 0.f;
  }
  float rd;
  rows_chol<NR>(A, rd, cb, nvp, lane);
  rows_store_strict<NR>(A, rd, Lm, nvp, lane);
  rows_fwd_rows<NR>(A, rd, lane);
  sync();
  float x = lane < nvp ? v[lane] : 0.f;
  x = rows_solve<NR>(A, rd, Lm, x, nvp, lane);
  if (lane < nvp) v[lane] = x;
  sync();
}

// --------------------------------------------------------------------------- collision
struct ConOut {
  float* S;
  int* ints;
  const Lds* L;
  int cap;
};
// Contact frame (mju_makeFrame) from the unit normal: rows n, t, b.  Phase A keeps only the
// normal in LDS and rebuilds the tangents where they are used (same arithmetic every time).
struct CFrame { V3 n, t, b; };
__device__ __forceinline__ CFrame cframe(V3 n) {
  CFrame f;
  f.n = n;
  V3 t = fabsf(n.y) < 0.5f ? V3{0, 1, 0} : V3{0, 0, 1};
  t = t - n * dot(n, t);
  f.t = t * (1.0f / fmaxf(norm(t), MINVAL));
  f.b = cross(n, f.t);
  return f;
}
// F^T v for the contact frame F rebuilt from the unit normal at np (the C pack carries the
// normals only)
__device__ __forceinline__ V3 frame_tv(const float* np, V3 v) {
  const CFrame F = cframe(v3(np));
  return F.n * v.x + F.t * v.y + F.b * v.z;
}
__device__ __forceinline__ void append(const ConOut& co, int key, int g1, int g2, float dist,
                                       V3 pos, V3 n) {
  int slot = atomicAdd(&co.ints[0], 1);
  if (slot >= co.cap) {
    atomicOr(&co.ints[3], 1);
    return;
  }
  const Lds& L = *co.L;
  int* Si = reinterpret_cast<int*>(co.S);
  Si[L.con_key + slot] = key;
  Si[L.con_g1 + slot] = g1;
  Si[L.con_g2 + slot] = g2;
  co.S[L.con_dist + slot] = dist;
  st3(co.S + L.con_pos + 3 * slot, pos);
  st3(co.S + L.con_n + 3 * slot, n);
}
__device__ __forceinline__ int plane_sphere(const ConOut& co, int key, int g1, int g2, V3 pp,
                                            V3 n, V3 c, float r, float margin) {
  float dist = dot(c - pp, n) - r;
  if (dist > margin) return 0;
  append(co, key, g1, g2, dist, c - n * (r + 0.5f * dist), n);
  return 1;
}
__device__ __forceinline__ int sphere_sphere(const ConOut& co, int key, int g1, int g2, V3 p1,
                                             float r1, V3 p2, float r2, float margin) {
  V3 dif = p2 - p1;
  float cd = norm(dif);
  float dist = cd - r1 - r2;
  if (dist > margin) return 0;
  V3 n = cd < MINVAL ? V3{1, 0, 0} : dif * (1.0f / cd);
  append(co, key, g1, g2, dist, p1 + n * (r1 + 0.5f * dist), n);
  return 1;
}
__device__ __forceinline__ float clamp01(float t) { return t < 0 ? 0 : (t > 1 ? 1 : t); }
__device__ __forceinline__ float clamp11(float t) { return t < -1 ? -1 : (t > 1 ? 1 : t); }
// Capsule-capsule as MuJoCo's mjc_CapsuleCapsule (engine_collision_primitive.c; restated
// from its published algorithm, mujoco_warp is absent here): segment parameters x1, x2 in
// [-1, 1] along the half-length-scaled axes A1, A2; the stationary point of the squared
// distance is clipped x1 first, then x2 (x1 re-solved and clipped), and the spheres at the
// two points collide.  Parallel axes give up to two contacts: each end of capsule 1 against
// its closest point on capsule 2, then, while fewer than two touch, each end of capsule 2.
// Parallel is MuJoCo's |det| < mjMINVAL, with det = ma mc - mb^2 evaluated as |A1 x A2|^2
// (Lagrange's identity): the difference form loses every digit to cancellation in fp32
// (rounding noise ~1e-7 ma mc, far above mjMINVAL), the cross-product form keeps
// exactly parallel axes below it in fp32 as in fp64.
__device__ __forceinline__ int capsule_capsule(const ConOut& co, int key, int g1, int g2, V3 p1,
                                               V3 A1, float r1, V3 p2, V3 A2, float r2,
                                               float margin) {
  const V3 dif = p1 - p2;
  const float ma = dot(A1, A1), mb = -dot(A1, A2), mc = dot(A2, A2);
  const float u = -dot(A1, dif), v = dot(A2, dif);
  const V3 cx = cross(A1, A2);
  const float det = dot(cx, cx);
  if (det >= MINVAL) {
    float x1 = (mc * u - mb * v) / det, x2 = (ma * v - mb * u) / det;
    if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
    else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
    if (x2 > 1) { x2 = 1; x1 = clamp11((u - mb) / ma); }
    else if (x2 < -1) { x2 = -1; x1 = clamp11((u + mb) / ma); }
    return sphere_sphere(co, key, g1, g2, p1 + A1 * x1, r1, p2 + A2 * x2, r2, margin);
  }
  int n = sphere_sphere(co, key, g1, g2, p1 + A1, r1, p2 + A2 * clamp11((v - mb) / mc), r2, margin);
  n += sphere_sphere(co, key + n, g1, g2, p1 - A1, r1, p2 + A2 * clamp11((v + mb) / mc), r2, margin);
  if (n >= 2) return n;
  n += sphere_sphere(co, key + n, g1, g2, p1 + A1 * clamp11((u - mb) / ma), r1, p2 + A2, r2, margin);
  if (n >= 2) return n;
  n += sphere_sphere(co, key + n, g1, g2, p1 + A1 * clamp11((u + mb) / ma), r1, p2 - A2, r2, margin);
  return n;
}
__device__ __forceinline__ void seg_seg(V3 a0, V3 a1, V3 b0, V3 b1, V3* pa, V3* pb) {
  V3 u = a1 - a0, v = b1 - b0, wv = a0 - b0;
  float a = dot(u, u), b = dot(u, v), c = dot(v, v), dd = dot(u, wv), e = dot(v, wv);
  float den = a * c - b * b, s, t;
  if (a < MINVAL && c < MINVAL) { s = t = 0; }
  else if (a < MINVAL) { s = 0; t = clamp01(e / c); }
  else if (c < MINVAL) { t = 0; s = clamp01(-dd / a); }
  else {
    s = den > MINVAL * a * c ? (b * e - c * dd) / den : 0;
    s = clamp01(s);
    t = (b * s + e) / c;
    if (t < 0) { t = 0; s = clamp01(-dd / a); }
    else if (t > 1) { t = 1; s = clamp01((b - dd) / a); }
  }
  *pa = a0 + u * s;
  *pb = b0 + v * t;
}


// Heightfield frame (static body) and the sphere-vs-hfield narrowphase.  The surface is the
// piecewise-linear interpolation of the elevation grid, two triangles per cell (p00 p10
// p11 / p00 p11 p01); the contact is the deepest closest-point over the triangles of the
// cells under the sphere footprint (oracle/oracle.c col_hfield_sphere, same arithmetic in
// fp32).  Row r spans y, column c spans x, as MuJoCo lays out hfield data.
struct HFrame { V3 p; float R[9]; };
__device__ __forceinline__ HFrame hfield_frame(const DModel& m, const float* S, const Lds& L,
                                               const float* gpos, const float* gquat, int g) {
  HFrame f;
  const int b = m.geom_bodyid[g];
  const Q4 qb = q4(S + L.xquat + 4 * b);
  f.p = v3(S + L.xpos + 3 * b) + qrot(qb, v3(gpos + 3 * g));
  qmat(f.R, qmul(qb, q4(gquat + 4 * g)));
  return f;
}
__device__ __forceinline__ int hfield_sphere(const ConOut& co, int key, int g1, int g2,
                                             const HFrame& F, const float* hdata,
                                             const float* hsize, int nr, int nc, V3 center,
                                             float r, float margin, int* trunc) {
  const V3 loc = mulTv(F.R, center - F.p);
  const float sx = hsize[0], sy = hsize[1], sz = hsize[2];
  const float dx = 2 * sx / (nc - 1), dy = 2 * sy / (nr - 1);
  int c0 = (int)floorf((loc.x - r + sx) / dx), c1 = (int)floorf((loc.x + r + sx) / dx);
  int r0 = (int)floorf((loc.y - r + sy) / dy), r1 = (int)floorf((loc.y + r + sy) / dy);
  if (c1 < 0 || r1 < 0 || c0 > nc - 2 || r0 > nr - 2) return 0;
  c0 = max(c0, 0); r0 = max(r0, 0);
  c1 = min(c1, nc - 2); r1 = min(r1, nr - 2);
  if ((c1 - c0 + 1) * (r1 - r0 + 1) > 64) { *trunc = 1; return 0; }  // footprint cap
  float best = 1e30f;
  V3 bestn = {0, 0, 1};
  bool found = false;
  for (int rr = r0; rr <= r1; rr++)
    for (int cc = c0; cc <= c1; cc++) {
      const float x0 = -sx + cc * dx, y0 = -sy + rr * dy;
      const float* row0 = hdata + rr * nc + cc;
      const V3 p00 = {x0, y0, row0[0] * sz}, p10 = {x0 + dx, y0, row0[1] * sz};
      const V3 p01 = {x0, y0 + dy, row0[nc] * sz}, p11 = {x0 + dx, y0 + dy, row0[nc + 1] * sz};
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const V3 a = p00, b = k ? p11 : p10, c = k ? p01 : p11;
        const V3 e1 = b - a, e2 = c - a;
        V3 n = cross(e1, e2);
        n = n * (1.0f / fmaxf(norm(n), MINVAL));
        const float sd = dot(loc - a, n);
        const V3 pp = loc - n * sd;
        const V3 v2 = pp - a;
        const float d00 = dot(e2, e2), d01 = dot(e2, e1), d11 = dot(e1, e1);
        const float d20 = dot(v2, e2), d21 = dot(v2, e1);
        const float den = d00 * d11 - d01 * d01;
        const float u = (d11 * d20 - d01 * d21) / den, vv = (d00 * d21 - d01 * d20) / den;
        V3 q;
        if (u >= 0 && vv >= 0 && u + vv <= 1) {
          q = pp;
        } else {
          float bd = 1e30f;
          q = a;
#pragma unroll
          for (int e = 0; e < 3; e++) {
            const V3 s0 = e == 0 ? a : (e == 1 ? b : c), s1 = e == 0 ? b : (e == 1 ? c : a);
            const V3 ab = s1 - s0;
            const float tt = clamp01(dot(loc - s0, ab) / fmaxf(dot(ab, ab), MINVAL));
            const V3 cp = s0 + ab * tt;
            const V3 df = loc - cp;
            const float dd = dot(df, df);
            if (dd < bd) { bd = dd; q = cp; }
          }
        }
        const V3 diff = loc - q;
        float dist = norm(diff);
        V3 nn;
        if (dist < MINVAL || sd < 0) { nn = n; dist = sd; }
        else { nn = diff * (1.0f / dist); }
        dist -= r;
        if (dist < best) { best = dist; bestn = nn; found = true; }
      }
    }
  if (!found || best > margin) return 0;
  const V3 nw = mulv(F.R, bestn);
  const V3 pw = mulv(F.R, loc - bestn * (r + 0.5f * best)) + F.p;
  append(co, key, g1, g2, best, pw, nw);
  return 1;
}

// Box narrowphase (terrain boxes welded to the world; oracle/oracle.c col_box_sphere /
// col_box_capsule, same arithmetic in fp64).  Signed distance of a box-frame point to the box
// of half sizes s (negative inside).
__device__ __forceinline__ float box_sd(V3 q, V3 s) {
  const float dx = fabsf(q.x) - s.x, dy = fabsf(q.y) - s.y, dz = fabsf(q.z) - s.z;
  const float ox = fmaxf(dx, 0.f), oy = fmaxf(dy, 0.f), oz = fmaxf(dz, 0.f);
  return sqrtf(ox * ox + oy * oy + oz * oz) + fminf(fmaxf(dx, fmaxf(dy, dz)), 0.f);
}
// Sphere (geom g1, centre `loc` in the box frame F) against the box (geom g2), MuJoCo's
// sphere-box contact: outside, the box point nearest the centre; inside, the face of least
// penetration.  Normal from the sphere to the box, position midway between the surfaces.
constexpr float kBoxFaceTie = 1e-5f;
__device__ __forceinline__ int box_sphere(const ConOut& co, int key, int g1, int g2,
                                          const HFrame& F, V3 s, V3 loc, float r, float margin) {
  const V3 cl = {fminf(fmaxf(loc.x, -s.x), s.x), fminf(fmaxf(loc.y, -s.y), s.y),
                 fminf(fmaxf(loc.z, -s.z), s.z)};
  const V3 dv = cl - loc;
  const float dist = norm(dv);
  if (dist - r > margin) return 0;
  V3 n, pos;
  float cd;
  if (dist > MINVAL) {
    n = dv * (1.0f / dist);
    pos = (cl + loc + n * r) * 0.5f;
    cd = dist - r;
  } else {
    // centre inside: the face of least penetration, faces within kBoxFaceTie of it tied and
    // taken in the order +z -z +x -x +y -y (terrain tops first).  A segment search inside
    // the box ends on such ties (box_capsule): the order keeps fp32 and fp64 on one face.
    const float f[6] = {s.z - loc.z, loc.z + s.z, s.x - loc.x, loc.x + s.x, s.y - loc.y, loc.y + s.y};
    float least = f[0];
#pragma unroll
    for (int i = 1; i < 6; i++) least = fminf(least, f[i]);
    int k = 5;
#pragma unroll
    for (int i = 4; i >= 0; i--)
      if (f[i] <= least + kBoxFaceTie) k = i;
    const float sg = (k & 1) ? 1.f : -1.f;  // a + face pushes the sphere out along +axis
    const int ax = k < 2 ? 2 : (k < 4 ? 0 : 1);
    n = {ax == 0 ? sg : 0.f, ax == 1 ? sg : 0.f, ax == 2 ? sg : 0.f};
    pos = loc + n * (0.5f * (r - f[k]));
    cd = -f[k] - r;
  }
  append(co, key, g1, g2, cd, F.p + mulv(F.R, pos), mulv(F.R, n));
  return 1;
}
// Capsule (geom g1: centre cw, unit axis aw, half length hl, radius r; world frame) against
// the box: sphere-box contacts at points of the capsule segment.  The signed box distance
// along the segment is convex; its minimiser (golden-section search, fixed iteration count)
// gives a contact only when it is deeper than both segment ends by kBoxMidEps (the segment
// crosses a box edge or corner), together with the deeper end; otherwise the two ends are
// the contact points (a capsule lying along a face), as plane-capsule.  At most 2 contacts.
constexpr float kBoxMidEps = 1e-4f;
constexpr int kBoxGolden = 28;
__device__ __forceinline__ int box_capsule(const ConOut& co, int key, int g1, int g2,
                                           const HFrame& F, V3 s, V3 cw, V3 aw, float hl,
                                           float r, float margin) {
  const V3 c = mulTv(F.R, cw - F.p), a = mulTv(F.R, aw);
  if (box_sd(c, s) - hl - r > margin) return 0;
  const V3 e0 = c - a * hl, e1 = c + a * hl;
  const float sd0 = box_sd(e0, s), sd1 = box_sd(e1, s);
  const float ig = 0.6180339887f;
  float lo = -hl, hi = hl;
  float x1 = hi - ig * (hi - lo), x2 = lo + ig * (hi - lo);
  float f1 = box_sd(c + a * x1, s), f2 = box_sd(c + a * x2, s);
  for (int it = 0; it < kBoxGolden; it++) {
    if (f1 <= f2) {
      hi = x2; x2 = x1; f2 = f1;
      x1 = hi - ig * (hi - lo);
      f1 = box_sd(c + a * x1, s);
    } else {
      lo = x1; x1 = x2; f1 = f2;
      x2 = lo + ig * (hi - lo);
      f2 = box_sd(c + a * x2, s);
    }
  }
  const float tm = 0.5f * (lo + hi);
  const V3 em = c + a * tm;
  int n = 0;
  if (box_sd(em, s) < fminf(sd0, sd1) - kBoxMidEps) {
    n += box_sphere(co, key, g1, g2, F, s, em, r, margin);
    n += box_sphere(co, key + n, g1, g2, F, s, sd0 <= sd1 ? e0 : e1, r, margin);
  } else {
    n += box_sphere(co, key, g1, g2, F, s, e0, r, margin);
    n += box_sphere(co, key + n, g1, g2, F, s, e1, r, margin);
  }
  return n;
}

// Box against box (separating axes), in the frame of box 1 (F1, half sizes s1): box 2 has
// centre c, axes b[0..2] (columns of R1^T R2) and half sizes s2.  Of the 15 axes (3 + 3 face
// normals, 9 edge crosses) the one of least penetration wins -- box 1 faces, then box 2
// faces, then edges, each later kind only when it separates more by kBoxFaceTie.  A face
// axis clips the other box's most anti-parallel face against the reference face's side
// planes (up to 8 points, those within the margin are contacts); an edge axis gives one
// contact between the two supporting edges.  Normals from geom 1 to geom 2.
__device__ __forceinline__ float vc(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
__device__ __forceinline__ V3 ev(int i) { return {i == 0 ? 1.f : 0.f, i == 1 ? 1.f : 0.f, i == 2 ? 1.f : 0.f}; }
__device__ __forceinline__ int box_face_clip(V3 sr, int k, float sgn, V3 c, const V3 (&b)[3], V3 si,
                                             float margin, V3 (&pt)[8], float (&dep)[8]) {
  int j = 0;
  float best = fabsf(vc(b[0], k));
  for (int jj = 1; jj < 3; jj++) {
    const float a = fabsf(vc(b[jj], k));
    if (a > best + kBoxFaceTie) { best = a; j = jj; }
  }
  const float fs = sgn * vc(b[j], k) > 0.f ? -1.f : 1.f;  // incident face looks back at box R
  const V3 fc = c + b[j] * (fs * vc(si, j));
  const V3 u = b[(j + 1) % 3] * vc(si, (j + 1) % 3), v = b[(j + 2) % 3] * vc(si, (j + 2) % 3);
  V3 poly[8], tmp[8];
  poly[0] = fc + u + v; poly[1] = fc - u + v; poly[2] = fc - u - v; poly[3] = fc + u - v;
  int np = 4;
  for (int a = 0; a < 3; a++) {
    if (a == k) continue;
    for (int side = -1; side <= 1; side += 2) {
      int nt = 0;
      for (int i = 0; i < np; i++) {
        const V3 P = poly[i], Q = poly[i + 1 < np ? i + 1 : 0];
        const float dp = side * vc(P, a) - vc(sr, a), dq = side * vc(Q, a) - vc(sr, a);
        if (dp <= 0.f) tmp[nt++] = P;
        if ((dp <= 0.f) != (dq <= 0.f)) tmp[nt++] = P + (Q - P) * (dp / (dp - dq));
      }
      np = nt;
      for (int i = 0; i < np; i++) poly[i] = tmp[i];
    }
  }
  int nc = 0;
  for (int i = 0; i < np; i++) {
    const float d = sgn * vc(poly[i], k) - vc(sr, k);
    if (d <= margin) { pt[nc] = poly[i]; dep[nc] = d; nc++; }
  }
  return nc;
}
__device__ __noinline__ int box_box(const ConOut& co, int key, int g1, int g2, const HFrame& F1,
                                    V3 s1, const HFrame& F2, V3 s2, float margin) {
  const V3 c = mulTv(F1.R, F2.p - F1.p);
  V3 b[3];
  for (int j = 0; j < 3; j++) b[j] = mulTv(F1.R, V3{F2.R[j], F2.R[3 + j], F2.R[6 + j]});
  float best = -1e30f;
  int kind = -1, ai = 0, aj = 0;
  V3 n = {0.f, 0.f, 1.f};
  for (int k = 0; k < 15; k++) {
    V3 L;
    int i = 0, j = 0;
    if (k < 3) { i = k; L = ev(k); }
    else if (k < 6) { j = k - 3; L = b[j]; }
    else { i = (k - 6) / 3; j = (k - 6) % 3; L = cross(ev(i), b[j]); }
    const float ln = norm(L);
    if (ln < 1e-6f) continue;
    L = L * (1.0f / ln);
    const float r1 = s1.x * fabsf(L.x) + s1.y * fabsf(L.y) + s1.z * fabsf(L.z);
    const float r2 = s2.x * fabsf(dot(L, b[0])) + s2.y * fabsf(dot(L, b[1])) + s2.z * fabsf(dot(L, b[2]));
    const float d = dot(L, c);
    const float sep = fabsf(d) - r1 - r2;
    if (sep > margin) return 0;
    const int kd = k < 3 ? 0 : (k < 6 ? 1 : 2);
    if (kind < 0 || sep > best + (kd > kind ? kBoxFaceTie : 0.f)) {
      best = sep; kind = kd; ai = i; aj = j;
      n = d < 0.f ? L * -1.f : L;
    }
  }
  V3 pt[8];
  float dep[8];
  int nc = 0;
  if (kind == 0) {
    nc = box_face_clip(s1, ai, vc(n, ai) < 0.f ? -1.f : 1.f, c, b, s2, margin, pt, dep);
  } else if (kind == 1) {
    // reference face on box 2: box 1 seen from box 2's frame, points mapped back
    V3 bt[3];
    for (int a = 0; a < 3; a++) bt[a] = {vc(b[0], a), vc(b[1], a), vc(b[2], a)};
    const V3 c2 = {-dot(b[0], c), -dot(b[1], c), -dot(b[2], c)};
    const float sg2 = dot(n, b[aj]) > 0.f ? -1.f : 1.f;  // box 2's face looking at box 1
    nc = box_face_clip(s2, aj, sg2, c2, bt, s1, margin, pt, dep);
    for (int q = 0; q < nc; q++) {
      const V3 w = pt[q];
      pt[q] = c + b[0] * w.x + b[1] * w.y + b[2] * w.z + n * dep[q];  // onto box 2's face side
    }
  } else {
    // supporting edges: box 1's most along +n, box 2's most along -n
    V3 p0 = {0.f, 0.f, 0.f}, q0 = c;
    for (int a = 0; a < 3; a++) {
      if (a != ai) p0 = p0 + ev(a) * (vc(n, a) > 0.f ? vc(s1, a) : -vc(s1, a));
      if (a != aj) q0 = q0 + b[a] * (dot(n, b[a]) > 0.f ? -vc(s2, a) : vc(s2, a));
    }
    const V3 ea = ev(ai) * vc(s1, ai), eb = b[aj] * vc(s2, aj);
    V3 pa, pb;
    seg_seg(p0 - ea, p0 + ea, q0 - eb, q0 + eb, &pa, &pb);
    const float d = dot(pb - pa, n);
    if (d <= margin) { pt[0] = pb; dep[0] = d; nc = 1; }
  }
  // points lie on box 2; the contact sits halfway back to box 1 along the normal
  for (int q = 0; q < nc; q++)
    append(co, key + q, g1, g2, dep[q], F1.p + mulv(F1.R, pt[q] - n * (0.5f * dep[q])), mulv(F1.R, n));
  return nc;
}

// --------------------------------------------------------------------------- impedance
__device__ __forceinline__ float impedance(const float* si, float pos, float margin) {
  float dmin = fminf(MAXIMP, fmaxf(MINIMP, si[0])), dmax = fminf(MAXIMP, fmaxf(MINIMP, si[1]));
  float width = fmaxf(0.f, si[2]), mid = fminf(1.f, fmaxf(MINIMP, si[3])), power = fmaxf(1.f, si[4]);
  if (dmin == dmax || width <= MINVAL) return 0.5f * (dmin + dmax);
  float x = fabsf(pos - margin) / width;
  if (x >= 1 || x <= 0) return x >= 1 ? dmax : dmin;
  float y;
  if (power == 1) y = x;
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1);
  else y = 1 - powf(1 - x, power) / powf(1 - mid, power - 1);
  return dmin + y * (dmax - dmin);
}

// reference stiffness / damping of a constraint row (mj_makeImpedance, solref > 0: time
// constant and damping ratio; solref <= 0: direct stiffness and damping)
__device__ __forceinline__ void solref_kb(const float* sref, const float* simp, float h, float& K,
                                          float& B) {
  const float dmax = fminf(MAXIMP, fmaxf(MINIMP, simp[1]));
  if (sref[0] > 0) {
    const float tc = fmaxf(sref[0], 2 * h), dr = sref[1];
    K = 1.0f / (dmax * dmax * tc * tc * dr * dr);
    B = 2.0f / (dmax * tc);
  } else {
    K = -sref[0] / (dmax * dmax);
    B = -sref[1] / dmax;
  }
}
// efc_cid row code: type (2 bits) | payload << 2; payload = contact index, or for joint
// limits joint | dof << 8
__device__ __forceinline__ int efc_code(int type, int payload) { return type | payload << 2; }

// --------------------------------------------------------------------------- specialisation
// ModelSpec<SP>: SP > 0 is the SP-th entry of specs.inc (scripts/gen_specs.py); its dims
// and the three phase carves are returned BY VALUE from constexpr functions, so every
// d.* bound and L.* LDS offset in the kernel folds to an immediate.  SP = 0 binds the
// run-time Params copies (generic kernels for any model).
// the specialisation table: csrc/specs.inc, or (a run-time JIT build, jit.hip) the one entry
// generated for a model no shipped entry matches
#ifndef MJX_SPECS_FILE
#define MJX_SPECS_FILE "specs.inc"
#endif
template <int SP> struct ModelSpec {
  static constexpr bool on = false;
  static constexpr Dims dims() { return Dims{}; }
};
#define MJX_SPEC(id, scene, ...)                                              \
  template <> struct ModelSpec<id> {                                          \
    static constexpr bool on = true;                                          \
    static constexpr Dims dims() { return Dims{__VA_ARGS__}; }                \
  };
#include MJX_SPECS_FILE
#undef MJX_SPEC
template <int SP> constexpr int spec_nr() { return nr_for_nv(ModelSpec<SP>::dims().nv); }
// box-box narrowphase compiled in: generic kernels, and specialisations with such pairs
template <int SP> constexpr bool kBoxBox = SP == 0 || ModelSpec<SP>::dims().nboxbox > 0;
// at most one contact per lane of the world's wave (every fast carve, nconmax <= 64): the
// contact loops of phases A and C are then the single lane-per-contact pass; a max carve past
// 64 contacts (sim.max_capacity: the reference's njmax bounds a world's contacts too) takes
// the multi-round forms (rank sort, contacts lane + 64 r)
template <int SP> constexpr bool kCon1 = SP != 0 && ModelSpec<SP>::dims().nconmax <= kWave;
// carve index kLdsJG: phase B at full capacity with J in global memory (make_lds jglobal)
constexpr int kLdsJG = 9;
template <int SP, int K> struct SpecLds {
  static constexpr Lds get() {
    constexpr Lds v = make_lds(ModelSpec<SP>::dims(), K == kLdsJG ? 1 : K, K == kLdsJG);
    return v;
  }
};
// `const auto& x = dims_of<SP>(P)`: a reference to Params for SP = 0, a constant
// temporary (folded) for SP > 0.
template <int SP>
__device__ __forceinline__ decltype(auto) dims_of(const Params* P) {
  if constexpr (SP > 0) return ModelSpec<SP>::dims();
  else return static_cast<const Dims&>(P->d);
}
template <int SP, int K>
__device__ __forceinline__ decltype(auto) lds_of(const Params* P) {
  if constexpr (SP > 0) return SpecLds<SP, K>::get();
  else if constexpr (K == kLdsJG) return static_cast<const Lds&>(P->LPJ);
  else return static_cast<const Lds&>(P->LP[K]);
}

// --------------------------------------------------------------------------- tree-sparse SPD
// A matrix whose pattern is the dof tree's (entry (i, j) != 0 only when one dof is an ancestor
// of the other: M, the implicit-integration matrix, and the Newton Hessian while every
// constraint row lies on one root-to-leaf chain) factors WITHOUT fill when children are
// eliminated before their parents (MuJoCo's L^T D L order).  The tree form of the
// register-row factor works in the reversed dof order (permuted index c = nvp-1-natural: pads
// first, leaves before their ancestors), where L[k][j] != 0 (k > j) iff natural(k) is an
// ancestor of natural(j).  For each 4-column block the trailing columns that block touches
// are a compile-time bit mask (the union of the block columns' ancestors), so the trailing
// update skips the structural zeros: 280 instead of 576 FMAs per lane for G1, 100 instead of
// 160 for Go1.  Skipped terms are exact zeros in the dense sweep, so on the reversed matrix
// the result equals the dense factor bit for bit.
struct TreeChol {
  bool on;
  uint64_t trail[16];  // per block b: permuted columns k >= 4b+4 with L[k][4b..4b+3] != 0
  uint32_t inblk[16];  // per block b: bit 4t+u set when L[4b+u][4b+t] != 0 (t < u)
};
constexpr TreeChol make_tree_chol(const int* par, int nv) {
  TreeChol t{};
  const int nvp = (nv + 3) & ~3;
  if (nv < 1 || nvp > 64) return t;
  for (int i = 0; i < nv; i++)
    if (par[i] >= i || par[i] < -1) return t;  // parents precede children
  t.on = true;
  for (int c = 0; c < nvp; c++) {
    const int n = nvp - 1 - c;
    if (n >= nv) continue;  // padding dof: identity row and column
    const int b = c >> 2;
    for (int a = par[n]; a >= 0; a = par[a]) {
      const int k = nvp - 1 - a;  // an ancestor's permuted index exceeds c
      if (k >= 4 * b + 4) t.trail[b] |= 1ull << k;
      else t.inblk[b] |= 1u << (4 * (c & 3) + (k & 3));
    }
  }
  return t;
}
template <int SP> struct SpecTree {
  static constexpr TreeChol get() { return TreeChol{}; }
  static constexpr int npar = 0;
  static constexpr int par[1] = {-1};
};
#define MJX_SPEC_TREE(id, ...)                                                \
  template <> struct SpecTree<id> {                                           \
    static constexpr int par[] = {__VA_ARGS__};                               \
    static constexpr int npar = sizeof(par) / sizeof(int);                    \
    static constexpr TreeChol get() { return make_tree_chol(par, npar); }     \
  };
#include MJX_SPECS_FILE
#undef MJX_SPEC_TREE
// which carve roles a specialisation serves (bit 0 fast, bit 1 max / re-solve): kernels of
// the other role are not compiled for it (phase_kernel returns null; the generic stand in)
template <int SP> struct SpecRole { static constexpr int mask = 3; };
#define MJX_SPEC_ROLE(id, m)                                                  \
  template <> struct SpecRole<id> { static constexpr int mask = m; };
#include MJX_SPECS_FILE
#undef MJX_SPEC_ROLE
// the tree form is compiled for a specialisation whose dof tree is known and matches its nv
template <int SP> constexpr bool kTree =
    SP > 0 && SpecTree<SP>::npar == ModelSpec<SP>::dims().nv && SpecTree<SP>::get().on;

// Register rows of the reversed matrix: lane i holds row nvp-1-i of Mm (row stride nvp, the
// natural order), columns reversed; lanes >= nvp identity.  The reversed lower triangle is
// the natural UPPER one: Mm must hold the full symmetric matrix (tiles_store_sym).
template <int NR>
__device__ __forceinline__ void rows_load_rev(float (&A)[NR], const float* Mm, int nvp, int lane) {
  const int row = lane < nvp ? nvp - 1 - lane : 0;
#pragma unroll
  for (int c = 0; c < NR; c += 4) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nvp) v = ld4(Mm + row * nvp + (nvp - 4 - c));
    A[c] = v.w; A[c + 1] = v.z; A[c + 2] = v.y; A[c + 3] = v.x;
  }
  if (NR > nvp || kWave > NR) {
    const int ln = opaque_lane(lane);
    const bool pad = ln >= nvp;
#pragma unroll
    for (int c = 0; c < NR; c++) A[c] = pad ? (c == ln ? 1.f : 0.f) : A[c];
  }
}
// rows_chol on the reversed matrix of a tree-pattern SPD matrix: the same blocked sweep with
// the structurally-zero in-block updates and trailing columns left out.  One instantiation
// per column block, so each block's masks are compile-time immediates.
template <int NR, int SP, int J0>
__device__ __forceinline__ void rows_chol_tree_blk(float (&A)[NR], float& rdiag, float* cb, int lane) {
  if constexpr (J0 < NR) {
    constexpr uint32_t ib = J0 < 64 ? SpecTree<SP>::get().inblk[J0 >> 2] : 0u;
    constexpr uint64_t tr = J0 < 64 ? SpecTree<SP>::get().trail[J0 >> 2] : 0ull;
    const int ln = opaque_lane(lane);
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = J0 + t;
      const float r = __builtin_amdgcn_rsqf(fmaxf(rl(A[j], j), MINVAL));
      A[j] *= r;
      rdiag = ln == j ? r : rdiag;
#pragma unroll
      for (int u = t + 1; u < 4; u++)
        if ((ib >> (4 * t + u)) & 1u) A[J0 + u] = fmaf(-A[j], rl(A[j], J0 + u), A[J0 + u]);
    }
    if constexpr (tr != 0ull) {
      st4v(cb + 4 * lane, make_float4(A[J0], A[J0 + 1], A[J0 + 2], A[J0 + 3]));
      sync();
#pragma unroll
      for (int k0 = J0 + 4; k0 < NR; k0 += 4) {
        if (((tr >> k0) & 0xfull) == 0ull) continue;
        float4 c[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
          if ((tr >> (k0 + u)) & 1ull) c[u] = ld4(cb + 4 * (k0 + u));
#pragma unroll
        for (int u = 0; u < 4; u++)
          if ((tr >> (k0 + u)) & 1ull)
            A[k0 + u] = fmaf(-A[J0 + 3], c[u].w, fmaf(-A[J0 + 2], c[u].z,
                        fmaf(-A[J0 + 1], c[u].y, fmaf(-A[J0], c[u].x, A[k0 + u]))));
      }
      sync();
    }
    rows_chol_tree_blk<NR, SP, J0 + 4>(A, rdiag, cb, lane);
  }
}
template <int NR, int SP>
__device__ __forceinline__ void rows_chol_tree(float (&A)[NR], float& rdiag, float* cb, int lane) {
  static_assert(NR % 4 == 0, "register rows come in column blocks of 4");
  rdiag = 1.f;
  rows_chol_tree_blk<NR, SP, 0>(A, rdiag, cb, lane);
}
// spd_factor_solve for a tree-pattern matrix: factor of the reversed matrix into Lm (reversed
// order), v solved in place (natural order in LDS).
template <int NR, int SP>
__device__ __forceinline__ void spd_factor_solve_tree(const float* Mm, float* Lm, float* v, float* cb,
                                                      int nvp, int lane) {
  float A[NR];
  rows_load_rev<NR>(A, Mm, nvp, lane);
  float rd;
  rows_chol_tree<NR, SP>(A, rd, cb, lane);
  rows_store_strict<NR>(A, rd, Lm, nvp, lane);
  rows_fwd_rows<NR>(A, rd, lane);
  sync();
  const int pl = nvp - 1 - lane;  // this lane's natural index (lanes < nvp)
  float x = lane < nvp ? v[pl] : 0.f;
  x = rows_solve<NR>(A, rd, Lm, x, nvp, lane);
  sync();
  if (lane < nvp) v[pl] = x;
  sync();
}

// --------------------------------------------------------------------------- kernels
// One substep = three launches, each holding only its own working set in LDS (more
// resident worlds per CU); hand-off through the per-world global scratch P->gscr, laid out
// with the full carve P->LG:
//   PH 0 (A): kinematics, com, CRB/M, velocity/RNE/actuation, smooth solve, subtree
//             momenta, pos/vel sensors, collision, contact parameters, constraint rows
//             (J rows written straight to the scratch);
//   PH 1 (B): Newton solver;
//   PH 2 (C): post-constraint acceleration, acc-stage sensors, contact forces, integration.
__device__ __forceinline__ void cp4(float* dst, const float* src, int n, int lane) {
  for (int i = 4 * lane; i < n; i += 4 * kWave) st4v(dst + i, ld4(src + i));
}
// Bulk global->LDS copy of a phase's input pack by LDS-DMA (global_load_lds_dwordx4: each
// wave-instruction lands 1 KiB at the wave-uniform LDS base + 16*lane, no VGPR staging), so
// the whole pack is in flight at once; the caller waits with lds_dma_wait() before reading.
// n is a multiple of 4 floats and dst/src are 16-byte aligned.
typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* glob_void_t;
__device__ __forceinline__ void cp_pack(float* __restrict__ dst, const float* __restrict__ src,
                                        int n, int lane) {
  for (int i0 = 0; i0 < n; i0 += 4 * kWave)
    if (i0 + 4 * lane < n)
      __builtin_amdgcn_global_load_lds((glob_void_t)(src + i0 + 4 * lane), (lds_void_t)(dst + i0),
                                       16, 0, 0);
}
// Global -> LDS copy of n floats (any alignment) by 4-byte LDS-DMA, lane per float.
__device__ __forceinline__ void dma_row(float* dst, const float* src, int n, int lane) {
  for (int i0 = 0; i0 < n; i0 += kWave)
    if (i0 + lane < n)
      __builtin_amdgcn_global_load_lds((glob_void_t)(src + i0 + lane), (lds_void_t)(dst + i0), 4, 0, 0);
}
// the same through L2 only (sc0 | sc1: past the vector L1), for state a phase earlier in the
// same launch stored (the L1 may still hold the lines that phase read before storing)
__device__ __forceinline__ void dma_row_l2(float* dst, const float* src, int n, int lane) {
  for (int i0 = 0; i0 < n; i0 += kWave)
    if (i0 + lane < n)
      __builtin_amdgcn_global_load_lds((glob_void_t)(src + i0 + lane), (lds_void_t)(dst + i0), 4, 0, 17);
}
__device__ __forceinline__ void lds_dma_wait() {
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ V3 point_vel(const float* S, const Lds& L, const DModel& m, int b, V3 p) {
  if (b <= 0) return {0.f, 0.f, 0.f};
  const float* cv = S + L.cvel + 6 * b;
  return v3(cv + 3) + cross(v3(cv), p - v3(S + L.subtree_com + 3 * m.body_rootid[b]));
}

// Per-lane model records, loaded once at phase entry: the tree passes then index registers
// instead of walking level_body -> body_* -> jnt_* chains of dependent global loads per
// level.  Lane i holds level-order body i (BodyRec), dof i (DofRec) and actuator i (ActRec);
// nbody, nv, nu <= 64 (mjx_model_create).  Only a body's first joint and five children are
// cached; further ones (rare) are read from the model arrays.
struct BodyRec {
  int b, p, lv, j0, jn, jt, qa, da, d0, dn, mocap, root, c0, cn, chp;
  uint64_t sub, dofs;  // subtree bodies (self included), dofs moving the body
  V3 pos, jpos, jaxis, ipos, inert;
  Q4 quat, iquat;
  float qp0, mass;
};
struct BodyPtrs {
  const float *pos, *quat, *ipos, *iquat, *mass, *inertia, *jpos, *jaxis, *qpos0;
};
__device__ __forceinline__ uint64_t u64_of(int lo, int hi) {
  return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32);
}
// the integer record (DModel::body_rec, level order): one dependent load level, then the
// body's and its first joint's floats
__device__ __forceinline__ BodyRec load_body(const DModel& m, const Dims& d, const BodyPtrs& P,
                                             int i) {
  (void)d;
  BodyRec r;
  const int4* rec = reinterpret_cast<const int4*>(m.body_rec + (size_t)kBodyRec * i);
  const int4 a = rec[0], b4 = rec[1], c4 = rec[2], e4 = rec[3], f4 = rec[4];
  r.b = a.x; r.p = a.y; r.lv = a.z; r.j0 = a.w;
  r.jn = b4.x; r.jt = b4.y; r.qa = b4.z; r.da = b4.w;
  r.d0 = c4.x; r.dn = c4.y; r.mocap = c4.z; r.root = c4.w;
  r.c0 = e4.x; r.cn = e4.y; r.chp = e4.z;
  r.sub = u64_of(f4.x, f4.y);
  r.dofs = u64_of(f4.z, f4.w);
  const int b = r.b;
  r.pos = v3(P.pos + 3 * b); r.quat = q4(P.quat + 4 * b);
  r.ipos = v3(P.ipos + 3 * b); r.iquat = q4(P.iquat + 4 * b);
  r.mass = P.mass[b]; r.inert = v3(P.inertia + 3 * b);
  const int k = r.jn > 0 ? r.j0 : 0;
  r.jpos = v3(P.jpos + 3 * k); r.jaxis = v3(P.jaxis + 3 * k);
  r.qp0 = P.qpos0[r.qa];
  return r;
}
__device__ __forceinline__ int body_child(const DModel& m, const BodyRec& r, int t) {
  return t < 5 ? (r.chp >> (6 * t)) & 63 : m.body_child[r.c0 + t];
}
// joint k of body r: the cached first joint or a model read
struct JntRec { int jt, qa, da; V3 jpos, jaxis; float qp0; };
__device__ __forceinline__ JntRec jnt_of(const DModel& m, const BodyPtrs& P, const BodyRec& r,
                                         int k) {
  if (k == r.j0) return {r.jt, r.qa, r.da, r.jpos, r.jaxis, r.qp0};
  const int qa = m.jnt_qposadr[k];
  return {m.jnt_type[k], qa, m.jnt_dofadr[k], v3(P.jpos + 3 * k), v3(P.jaxis + 3 * k), P.qpos0[qa]};
}
struct BodyLite { int b, p, lv, d0, dn; uint64_t dofs; };
__device__ __forceinline__ BodyLite load_body_lite(const DModel& m, const Dims& d, int i) {
  (void)d;
  BodyLite r;
  const int4* rec = reinterpret_cast<const int4*>(m.body_rec + (size_t)kBodyRec * i);
  const int4 a = rec[0], c4 = rec[2], f4 = rec[4];
  r.b = a.x; r.p = a.y; r.lv = a.z;
  r.d0 = c4.x; r.dn = c4.y;
  r.dofs = u64_of(f4.z, f4.w);
  return r;
}
struct DofRec {
  int body, jt, qa, pbody, jd0, bd0;  // parent body, first dof of the joint / of the body
  uint64_t anc;
  float arm, damp, stiff, qs;
};
struct ActRec {
  int dof, qa, ctrllim, forcelim;
  float gear, gain, b0, b1, b2, fr0, fr1, cr0, cr1;
};
__device__ __forceinline__ ActRec load_act(const DModel& m, const float* gear, const float* gain,
                                           const float* bias, const float* frange,
                                           const float* crange, int u) {
  ActRec r;
  const int4 a = *reinterpret_cast<const int4*>(m.act_rec + (size_t)kActRec * u);
  r.dof = a.x; r.qa = a.y; r.ctrllim = a.z; r.forcelim = a.w;
  r.gear = gear[u]; r.gain = gain[3 * u];
  r.b0 = bias[3 * u]; r.b1 = bias[3 * u + 1]; r.b2 = bias[3 * u + 2];
  r.fr0 = frange[2 * u]; r.fr1 = frange[2 * u + 1];
  r.cr0 = crange[2 * u]; r.cr1 = crange[2 * u + 1];
  return r;
}
// contact bodies packed in one int (nbody <= 64): b1 | b2 << 8 | root(b1) << 16 | root(b2) << 24
__device__ __forceinline__ int cb_b1(int v) { return v & 255; }
__device__ __forceinline__ int cb_b2(int v) { return (v >> 8) & 255; }
__device__ __forceinline__ int cb_r1(int v) { return (v >> 16) & 255; }
__device__ __forceinline__ int cb_r2(int v) { return (v >> 24) & 255; }
__device__ __forceinline__ V3 point_vel_r(const float* S, const Lds& L, int b, int root, V3 p) {
  if (b <= 0) return {0.f, 0.f, 0.f};
  const float* cv = S + L.cvel + 6 * b;
  return v3(cv + 3) + cross(v3(cv), p - v3(S + L.subtree_com + 3 * root));
}

// mjSENS_CONTACT with one slot (sensor/contact_sensor.py:16-97, 472-533), one wave per
// world, lane = contact: every sensor the contact matches comes from two transposed geom
// masks (one load pair per contact, not one per sensor), then per sensor found =
// popcount(ballot), netforce = wave sums of the signed world-frame forces, and for mindist /
// maxforce / none the single selected contact is the wave argmin of its key (ties ->
// lowest contact index).
__device__ __forceinline__ void contact_sensors_wave(const float* S, const int* Si, const Lds& L,
                                                     const DModel& m, const Dims& d, float* sd,
                                                     int ncon, int maxmatch, bool all,
                                                     const Params* __restrict__ P, int lane) {
  const int c = lane;
  const bool valid = c < ncon;
  V3 fg = {0, 0, 0}, fc = {0, 0, 0};
  float dist = 0.f;
  // the sensors this contact matches, all at once: bit k of m1 (m2) = sensor k with the
  // contact's geom 1 (geom 2) as its primary (geom_csmask1/2, host-derived)
  uint64_t m1 = 0, m2 = 0;
  if (valid) {
    const int g1 = Si[L.con_g1 + c], g2 = Si[L.con_g2 + c];
    m1 = m.geom_csmask1[g1] & m.geom_csmask2[g2];
    m2 = m.geom_csmask1[g2] & m.geom_csmask2[g1];
    if (all) {  // (before the last substep only found counts are computed: no forces)
      dist = S[L.con_dist + c];
      const int r0 = Si[L.con_efc + c];
      if (Si[L.con_dim + c] == 1) {
        fc.x = S[L.efc_force + r0];
      } else {
        float e0 = S[L.efc_force + r0], e1 = S[L.efc_force + r0 + 1];
        float e2 = S[L.efc_force + r0 + 2], e3 = S[L.efc_force + r0 + 3];
        fc = {e0 + e1 + e2 + e3, (e0 - e1) * S[L.con_mu + 2 * c], (e2 - e3) * S[L.con_mu + 2 * c + 1]};
      }
      fg = frame_tv(S + L.con_n + 3 * c, fc);
    }
  }
  // the sensors' descriptors, lane k = k-th single-slot contact sensor (ncsens <= 64): the
  // loop below reads them with v_readlane instead of a dependent scalar-load chain per sensor
  const int ncs = m.ncsens;
  int dbits = 0, dred = 0, dadr = 0, ddim = 0;
  if (lane < ncs) {
    const int s = m.cs_sensor[lane];
    dbits = m.sensor_intprm[3 * s];
    dred = m.sensor_intprm[3 * s + 1];
    dadr = m.sensor_adr[s];
    ddim = m.sensor_dim[s];
  }
  // found-only sensors (data = found, one slot: Go1's 26 non-foot touch sensors): the count
  // of matching contacts is the output whatever the reduce, so each costs one ballot and
  // popcount kept in its own lane, and all of them go out in one store at the end
  const bool fonly = lane < ncs && dbits == 1 && ddim == 1;
  // contact_sensor_maxmatch below the contact count: a sensor keeps its first maxmatch
  // matching contacts (lanes), as the serial form does
  const bool mtrunc = maxmatch < ncon;
  const uint64_t below = (1ull << lane) - 1ull;
  const uint64_t mm = m1 | m2;
  float fcount = 0.f;
  uint64_t rest = __ballot(lane < ncs && !fonly);
  for (uint64_t fo = __ballot(fonly); fo; fo &= fo - 1) {
    const int k = __ffsll((long long)fo) - 1;
    const float f = (float)min(__popcll(__ballot((mm >> k) & 1ull)), maxmatch);
    fcount = lane == k ? f : fcount;
  }
  if (fonly) sd[dadr] = fcount;
  for (; rest; rest &= rest - 1) {
    const int k = __ffsll((long long)rest) - 1;
    const int bits = __builtin_amdgcn_readlane(dbits, k), reduce = __builtin_amdgcn_readlane(dred, k);
    const int adr = __builtin_amdgcn_readlane(dadr, k), dim = __builtin_amdgcn_readlane(ddim, k);
    if (!all) {  // not the last substep: only a contact air time's found count is read
      bool air = false;
      for (int i = 0; i < P->nair; i++) air |= P->air_found[i] == adr;
      if (!air) continue;
    }
    float* out = sd + adr;
    bool a1 = (m1 >> k) & 1ull, a2 = (m2 >> k) & 1ull;
    if (mtrunc) {
      const bool keep = __popcll(__ballot(a1 || a2) & below) < maxmatch;
      a1 = a1 && keep;
      a2 = a2 && keep;
    }
    const bool match = a1 || a2;
    const unsigned long long bal = __ballot(match);
    const float found = (float)__popcll(bal);
    // every output element of the sensor in one store (lanes < dim <= 3): the zeros of
    // mjSENS_CONTACT's empty slot and the selected values at once
    float v = 0.f;
    if (reduce == REDUCE_NETFORCE) {
      const float sg = match ? (a1 ? 1.f : -1.f) : 0.f;
      const float nx = wave_sum(sg * fg.x), ny = wave_sum(sg * fg.y), nz = wave_sum(sg * fg.z);
      if (bits & 1) v = lane == 0 ? found : 0.f;
      else if (bits & 2) v = lane == 0 ? nx : lane == 1 ? ny : lane == 2 ? nz : 0.f;
    } else {
      // one slot: the matching contact with the smallest key (ties -> lowest contact index)
      int sel = -1;
      if (reduce == REDUCE_NONE) {
        sel = bal ? __ffsll((long long)bal) - 1 : -1;  // key = contact index
      } else {
        float key = reduce == REDUCE_MINDIST ? dist : -sqrtf(fc.x * fc.x + fc.y * fc.y + fc.z * fc.z);
        if (!match) key = FLT_MAX;
        const float kmin = wave_min(key);
        const unsigned long long win = __ballot(match && key == kmin);
        sel = win ? __ffsll((long long)win) - 1 : -1;
      }
      if (sel >= 0) {
        const int cs = sel;
        const float sg = rl(a1 ? 1.f : -1.f, cs);
        const int t = lane < 3 ? lane : 0;
        if (bits & 1) v = lane == 0 ? found : 0.f;
        else if (bits & 8) v = lane == 0 ? rl(dist, cs) : 0.f;
        else if (bits & 16) v = lane < 3 ? S[L.con_pos + 3 * cs + t] : 0.f;
        else if (bits & 32) v = lane < 3 ? sg * S[L.con_n + 3 * cs + t] : 0.f;
        else if (bits & 64) v = lane < 3 ? sg * vc(cframe(v3(S + L.con_n + 3 * cs)).t, t) : 0.f;
        else if (bits & 2) {
          const float fx = rl(fc.x, cs), fy = rl(fc.y, cs), fz = rl(fc.z, cs);
          v = lane == 0 ? fx : lane == 1 ? fy : lane == 2 ? fz : 0.f;
        }
      }
    }
    if (lane < dim) out[lane] = v;
  }
}

// Worlds [w0, w1) -- one split of the batch (launch_step).  `sel` & 0xff selects that
// split's Newton work-list segments; in phases A and C, sel >> 8 = row class + 1 restricts
// the launch to that class's worlds (0: every world).
// Phase B at most 168 registers (3 waves / SIMD): the Newton kernel's allocation drifts with
// small code changes (G1 161 -> 177 with the LTR Hessian; no spill at 168) and the bulk row
// class's residency is set by it.  Not for the generic NR 56 / 64 rows (they would spill).
// Phase A at most 168 registers too: with terrain collision (heightfields, box terrains) its
// natural allocation is 182-189 VGPRs (2 waves / SIMD, 8 worlds per CU) while its LDS admits 12;
// capped it spills a few dozen bytes per lane (-Rpass-analysis=kernel-resource-usage), as the
// chain kernel that inlines the same code already does.  The flat models sit at 126-135.
// "Lean" specialisations: a small-robot (NR <= 20) model without terrain collision whose phase
// carves all fit 16 worlds per CU (<= 10,240 B: Go1 at its 16 / 64 fast carve).  Their phase B
// and chain kernels are held to 128 VGPRs (4 waves / SIMD; naturally 145-147, capped they spill
// ~40 B per lane), so the LDS residency is the register residency too.  Elsewhere 4 waves
// would only add spill (Go1 at 24 / 96, whose phase-B carve admits 12 per CU: -0.5 %; rough
// Go1, whose chain inlines the box-box arrays: -20 %).
template <int SP>
constexpr bool lean_spec() {
  if constexpr (SP <= 0) {
    return false;
  } else {
    constexpr Dims d = ModelSpec<SP>::dims();
    return nr_for_nv(d.nv) <= 20 && d.nstatic == 0 && d.nboxbox == 0 &&
           make_lds(d, 0).total * 4 <= 10240 && make_lds(d, 1).total * 4 <= 10240 &&
           make_lds(d, 2).total * 4 <= 10240;
  }
}
template <int SP> constexpr bool kLean = lean_spec<SP>();
#define MJX_PHASE_ATTR __attribute__((amdgpu_waves_per_eu(PH == 1 && kLean<SP> ? 4 : (PH == 1 || PH == 0) && NR <= 48 ? 3 : 1)))
#define MJX_PHASE_ATTR_B __attribute__((amdgpu_waves_per_eu(NR <= 48 ? 3 : 1)))
// LAT selects the latency form of phase B (step_newton_lat below): the same algorithm with
// more registers in flight, for the launch that holds the heavy worlds.
// LAT: bit 0 the latency form of phase B (else the throughput form), bit 1 (phase B only) the
// constraint Jacobian read from the B pack in global memory (carve kLdsJG)
template <int NR, int PH, int SP, int LAT>
__device__ __forceinline__ void step_body(float* __restrict__ S, const Params* __restrict__ P, int w0,
                                          int w1, int sel, int last, int integrate,
                                          const uint8_t* __restrict__ mask, const int bid) {
  const auto& d = dims_of<SP>(P);
  const Opt& o = P->o;
  const DModel& m = P->m;
  const DData& D = P->D;
  // phase B: `integrate` carries the Newton row class (0 = full capacity, k > 0 = LP[2 + k])
  constexpr bool JG = PH == 1 && (LAT & 2) != 0;
  const Lds& L = (PH == 1 && integrate > 0) ? P->LP[2 + integrate]
                                            : lds_of<SP, JG ? kLdsJG : PH>(P);
  const auto& LB = lds_of<SP, 1>(P);
  const auto& LC = lds_of<SP, 2>(P);
  if (sel & kSelPrio) __builtin_amdgcn_s_setprio(3);
  int w = w0 + bid;
  const int sel_arg = sel;  // (phase C's contact-sensor code has a local `sel`)
  (void)sel_arg;
  const int split = sel & 0xff;
  const int cls1 = (sel >> 8) & 0xff;
  if (sel & kSelOvf) {
    // overflow re-solve: workgroup i takes the i-th world phase A listed (parity kSelRPar)
    const int li = 2 * split + ((sel & kSelRPar) ? 1 : 0);
    if (bid >= min(P->ovf_n[li], P->ovf_cap)) return;
    w = P->ovf_list[(size_t)li * P->ovf_cap + bid];
  } else {
    if constexpr (PH == 1) {
      // Newton by row class: workgroup i takes the i-th world of its class's list
      // (classify_kernel: rows descending, masked worlds only)
      if (P->nrowclass > 0 && integrate >= 0) {  // integrate < 0: every world, full carve
        const int* seg = P->wl_seg + 2 * ((kRowClasses + 1) * split + integrate);
        if (bid >= seg[1]) return;
        w = P->wl_list[seg[0] + bid];
      }
    }
    if constexpr (PH == 0 || PH == 2) {
      // phase C of one row class right behind that class's Newton launch, and phase A of the
      // next substep for the same worlds (the class lists stay valid until the next classify)
      if (cls1) {
        const int* seg = P->wl_seg + 2 * ((kRowClasses + 1) * split + cls1 - 1);
        if (bid >= seg[1]) return;
        w = P->wl_list[seg[0] + bid];
      }
    }
  }
  if (w >= w1) return;
  if (mask && !mask[w]) return;  // masked forward: only the selected worlds
  // a world listed for the overflow re-solve this substep skips this carve's B and C (the
  // class lists already leave it out; the all-world launches check)
  // (list-driven launches -- a Newton row class, a class pipeline's C -- never see them:
  // classify_kernel left them out, and their one extra dependent load stays off the chain)
  if (PH != 0 && P->ovf_resolve && !(sel & kSelOvf) && !cls1 &&
      !(PH == 1 && P->nrowclass > 0 && integrate >= 0) && P->ovf_flag[w])
    return;
  // ... and a range chain's next phase A (models without row classes: step_chain over every
  // world of a batch range) skips it too: the re-solve chain runs that world's next A
  if (PH == 0 && (sel & kSelFusedA) && !cls1 && P->ovf_resolve && P->ovf_flag[w]) return;
  float* gw = P->gscr + (size_t)w * P->gstride;  // [B pack | C pack]
  float* gc = gw + P->gC;
  float* gf = gw + P->gF;  // implicit-integration factor (phase A writes, phase C reads)
  (void)LB; (void)LC; (void)gc;
  const int lane = threadIdx.x;
  int* Si = reinterpret_cast<int*>(S);
  int* ints = Si + L.ints;
  const int nv = d.nv, nb = d.nbody, nq = d.nq, nu = d.nu;
  const int nvp = (nv + 3) & ~3;
  const int nvq = (nvp + 3) & ~3;  // copy length of an nvp vector region
  const float h = o.timestep;
  (void)nq; (void)nu; (void)h;
#ifdef MJX_STAMPS
  const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long stamp_prev = __builtin_amdgcn_s_memtime();
  unsigned long long sub_prev = stamp_prev;
  unsigned long long stamp_acc[48];
#pragma unroll
  for (int k_ = 0; k_ < 48; k_++) stamp_acc[k_] = 0;
#endif
  const float* body_pos = MF(body_pos);
  const float* body_quat = MF(body_quat);
  const float* body_ipos = MF(body_ipos);
  const float* body_iquat = MF(body_iquat);
  const float* body_mass = MF(body_mass);
  const float* body_inertia = MF(body_inertia);
  const float* jnt_pos = MF(jnt_pos);
  const float* jnt_axis = MF(jnt_axis);
  const float* qpos0 = MF(qpos0);
  (void)body_pos; (void)body_quat; (void)body_ipos; (void)body_iquat; (void)body_mass;
  (void)body_inertia; (void)jnt_pos; (void)jnt_axis; (void)qpos0;

  if constexpr (PH == 0) {
    // ----------------------------------------------------------- phase A
    // Preamble: every independent global read is in flight before the first wait -- state
    // rows go straight into LDS (LDS-DMA), model records into registers, then one wait
    // (copied loop by loop, each load-then-LDS-store would wait out a global latency).
    for (int i = lane; i < nvp; i += kWave) {
      if (i >= nv) S[L.qvel + i] = 0.f;  // DMA fills i < nv
    }
    if (sel & kSelFusedA) {  // step_chain: phase C stored this state in the same launch
      dma_row_l2(S + L.qpos, D.qpos + (size_t)w * nq, nq, lane);
      dma_row_l2(S + L.qvel, D.qvel + (size_t)w * nv, nv, lane);
    } else {
      dma_row(S + L.qpos, D.qpos + (size_t)w * nq, nq, lane);
      dma_row(S + L.qvel, D.qvel + (size_t)w * nv, nv, lane);
    }
    // lane-aligned inputs stay in registers (lane u: ctrl[u], lane i: qfrc_applied[i])
    const float ctrl_u = lane < nu ? D.ctrl[(size_t)w * nu + lane] : 0.f;
    const float qapp_i = lane < nv ? D.qfrc_applied[(size_t)w * nv + lane] : 0.f;
    SUBSTAMP(15);
    float* Jg = gw + LB.efc_J;
    const BodyPtrs BP{body_pos, body_quat, body_ipos, body_iquat, body_mass, body_inertia,
                      jnt_pos, jnt_axis, qpos0};
    const BodyRec B = load_body(m, d, BP, min(lane, nb - 1));
#ifdef MJX_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
#endif
    SUBSTAMP(16);
    const bool bl = lane < nb;  // this lane holds a body record
    DofRec Dr;
    {
      const int i = min(lane, max(nv - 1, 0));
      const float* arm = MF(dof_armature);
      const float* damping = MF(dof_damping);
      const float* jstiff = MF(jnt_stiffness);
      const float* qspring = MF(qpos_spring);
      const int4* rec = reinterpret_cast<const int4*>(m.dof_rec + (size_t)kDofRec * i);
      const int4 a = rec[0], b4 = rec[1], c4 = rec[2];
      Dr.body = a.x; Dr.jt = a.y; Dr.qa = a.z; Dr.pbody = a.w;
      Dr.jd0 = b4.x; Dr.bd0 = b4.y;
      const int j = b4.z;
      Dr.anc = u64_of(c4.x, c4.y);
      Dr.arm = arm[i]; Dr.damp = damping[i]; Dr.stiff = jstiff[j]; Dr.qs = qspring[Dr.qa];
    }
#ifdef MJX_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
#endif
    SUBSTAMP(17);
    const ActRec Ar = load_act(m, MF(actuator_gear), MF(actuator_gainprm), MF(actuator_biasprm),
                               MF(actuator_forcerange), MF(actuator_ctrlrange),
                               min(lane, max(nu - 1, 0)));
    int any_xfrc = 0;
    for (int i = lane; i < 6 * nb; i += kWave) any_xfrc |= D.xfrc_applied[(size_t)w * 6 * nb + i] != 0.f;
    any_xfrc = __any(any_xfrc);
    lds_dma_wait();
    sync();
    SUBSTAMP(13);
    // =========================================================== kinematics
    // (1) lane per body: the body frame in its parent's frame (body offset, then its
    //     joints) and the joint anchors / axes in that frame; free-joint, mocap and world
    //     bodies are absolute (world) frames;
    // (2) pointer jumping over the tree: T(b) <- T(anc) o T(b), anc <- anc(anc), until every
    //     chain reaches an absolute frame -- ceil(log2(depth)) rounds of one LDS round trip
    //     instead of one per tree level;
    // (3) after the body frames: anchors / axes to the world by the parent frame.
    // A free body's tree is built about the free body's own position (root-relative frame)
    // and moved to the world only after cinert / cdof: their offsets (xipos - subtree_com,
    // subtree_com - anchor) are then differences of O(1 m) numbers, not of world
    // coordinates up to ~100 m from the origin (fp32 ulp(80) = 7.6e-6 m, which a light
    // wrist's mass-matrix entry, a difference of O(m d^2) terms, amplifies to 1e-3 relative).
    int* par = Si + L.efc_cid;  // scratch ancestor pointers (the row block is dead until rows)
    bool absb = false;
    V3 proot = {0.f, 0.f, 0.f};  // free body: its world position (added back below)
    V3 kpos = {0.f, 0.f, 0.f};
    Q4 kq = {1.f, 0.f, 0.f, 0.f};
    if (bl) {
      const int b = B.b;
      kpos = B.pos;
      kq = B.quat;
      if (b == 0) {
        kpos = {0.f, 0.f, 0.f};
        kq = {1.f, 0.f, 0.f, 0.f};
        absb = true;
      }
      if (B.mocap >= 0) {
        kpos = v3(D.mocap_pos + ((size_t)w * d.nmocap + B.mocap) * 3);
        kq = q4(D.mocap_quat + ((size_t)w * d.nmocap + B.mocap) * 4);
        absb = true;
      }
      for (int k = B.j0; k < B.j0 + B.jn; k++) {
        const JntRec J = jnt_of(m, BP, B, k);
        const int a = J.qa;
        float R[9];
        if (J.jt == JNT_FREE) {  // MuJoCo: the only joint of a top-level body
          proot = v3(S + L.qpos + a);
          kpos = {0.f, 0.f, 0.f};
          kq = qnorm(q4(S + L.qpos + a + 3));
          st3(S + L.xanchor + 3 * k, kpos);
          qmat(R, kq);
          st3(S + L.xaxis + 3 * k, mulv(R, J.jaxis));
          absb = true;
          continue;
        }
        qmat(R, kq);
        const V3 anchor = mulv(R, J.jpos) + kpos;
        const V3 axis = mulv(R, J.jaxis);
        st3(S + L.xanchor + 3 * k, anchor);  // parent frame, to the world in (3)
        st3(S + L.xaxis + 3 * k, axis);
        if (J.jt == JNT_HINGE) {
          kq = qmul(kq, qaxisangle(J.jaxis, S[L.qpos + a] - J.qp0));
          qmat(R, kq);
          kpos = anchor - mulv(R, J.jpos);
        } else if (J.jt == JNT_SLIDE) {
          kpos = kpos + axis * (S[L.qpos + a] - J.qp0);
        }
      }
      st3(S + L.xpos + 3 * b, kpos);
      st4(S + L.xquat + 4 * b, kq);
      par[b] = absb ? 0 : B.p;
    }
    sync();
    {
      int pa = bl ? par[B.b] : 0;
      while (__any(pa != 0)) {
        V3 ppos = {0.f, 0.f, 0.f};
        Q4 pq = {1.f, 0.f, 0.f, 0.f};
        int ppa = 0;
        if (pa != 0) {
          ppos = v3(S + L.xpos + 3 * pa);
          pq = q4(S + L.xquat + 4 * pa);
          ppa = par[pa];
        }
        sync();  // every lane's reads precede every lane's writes (one wave: LDS in order)
        if (pa != 0) {
          kpos = ppos + qrot(pq, kpos);
          kq = qmul(pq, kq);
          st3(S + L.xpos + 3 * B.b, kpos);
          st4(S + L.xquat + 4 * B.b, kq);
          par[B.b] = ppa;
          pa = ppa;
        }
        sync();
      }
    }
    if (bl) st4(S + L.xquat + 4 * B.b, qnorm(kq));
    sync();
    SUBSTAMP(14);
    // body rotations stay quaternions in LDS (xmat / ximat are formed where used)
    const Q4 xq = bl ? q4(S + L.xquat + 4 * B.b) : Q4{1.f, 0.f, 0.f, 0.f};
    if (bl) st3(S + L.xipos + 3 * B.b, v3(S + L.xpos + 3 * B.b) + qrot(xq, B.ipos));
    if (bl && !absb) {  // (3): joint anchors / axes from the parent frame to the world
      const Q4 qp = q4(S + L.xquat + 4 * B.p);
      const V3 pp = v3(S + L.xpos + 3 * B.p);
      for (int k = B.j0; k < B.j0 + B.jn; k++) {
        st3(S + L.xanchor + 3 * k, pp + qrot(qp, v3(S + L.xanchor + 3 * k)));
        st3(S + L.xaxis + 3 * k, qrot(qp, v3(S + L.xaxis + 3 * k)));
      }
    }
    STAMP(0);
    // =========================================================== com / cinert / cdof
    // Subtree sums as broadcast loops: lane b adds body c's term when c is in its subtree
    // (B.sub); every lane reads the same LDS address per c, no level-by-level syncs.
    float stm = 0.f;  // subtree mass of this lane's body
    {
      float* mx = S + L.crb;  // scratch [nb][4] = (m * xipos, m); crb is written below
      if (bl) {
        const V3 xi = v3(S + L.xipos + 3 * B.b);
        st4v(mx + 4 * B.b, make_float4(B.mass * xi.x, B.mass * xi.y, B.mass * xi.z, B.mass));
      }
      sync();
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
      for (int c = 0; c < nb; c++) {
        const float4 v = ld4(mx + 4 * c);
        const float f = (B.sub >> c) & 1ull ? 1.f : 0.f;
        acc.x = fmaf(f, v.x, acc.x); acc.y = fmaf(f, v.y, acc.y);
        acc.z = fmaf(f, v.z, acc.z); acc.w = fmaf(f, v.w, acc.w);
      }
      sync();
      if (bl) {
        const int b = B.b;
        stm = acc.w;
        const V3 c = acc.w > MINVAL ? V3{acc.x, acc.y, acc.z} * (1.0f / acc.w) : v3(S + L.xipos + 3 * b);
        st3(S + L.subtree_com + 3 * b, c);
      }
      sync();
    }
    if (bl) {
      const int b = B.b;
      float* c = S + L.cinert + 10 * b;
      if (b == 0) {
        for (int i = 0; i < 10; i++) c[i] = 0;
      } else {
      V3 off = v3(S + L.subtree_com + 3 * B.root);
      float R[9];  // ximat
      qmat(R, qmul(xq, B.iquat));
      const float I[3] = {B.inert.x, B.inert.y, B.inert.z};
      float full[9];
#pragma unroll
      for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
          full[3 * i + j] = R[3 * i] * I[0] * R[3 * j] + R[3 * i + 1] * I[1] * R[3 * j + 1] +
                            R[3 * i + 2] * I[2] * R[3 * j + 2];
      V3 dv = v3(S + L.xipos + 3 * b) - off;
      float ms = B.mass, dd = dot(dv, dv);
      c[0] = full[0] + ms * (dd - dv.x * dv.x);
      c[1] = full[4] + ms * (dd - dv.y * dv.y);
      c[2] = full[8] + ms * (dd - dv.z * dv.z);
      c[3] = full[1] - ms * dv.x * dv.y;
      c[4] = full[2] - ms * dv.x * dv.z;
      c[5] = full[5] - ms * dv.y * dv.z;
      c[6] = ms * dv.x; c[7] = ms * dv.y; c[8] = ms * dv.z; c[9] = ms;
      }
    }
    // cdof: lane per body over its joints
    for (int k = B.j0; bl && k < B.j0 + B.jn; k++) {
      const JntRec J = jnt_of(m, BP, B, k);
      const int dof = J.da;
      V3 rel = v3(S + L.subtree_com + 3 * B.root) - v3(S + L.xanchor + 3 * k);
      const int t = J.jt;
      if (t == JNT_FREE) {
        for (int i = 0; i < 3; i++) {
          float* c = S + L.cdof + 6 * (dof + i);
          for (int j = 0; j < 6; j++) c[j] = 0;
          c[3 + i] = 1;
        }
        float R[9];
        qmat(R, xq);
        for (int i = 0; i < 3; i++) {
          float* c = S + L.cdof + 6 * (dof + 3 + i);
          V3 ax = {R[i], R[3 + i], R[6 + i]};
          st3(c, ax);
          st3(c + 3, cross(ax, rel));
        }
      } else if (t == JNT_HINGE) {
        float* c = S + L.cdof + 6 * dof;
        V3 ax = v3(S + L.xaxis + 3 * k);
        st3(c, ax);
        st3(c + 3, cross(ax, rel));
      } else if (t == JNT_SLIDE) {
        float* c = S + L.cdof + 6 * dof;
        c[0] = c[1] = c[2] = 0;
        st3(c + 3, v3(S + L.xaxis + 3 * k));
      }
    }
    sync();
    {  // root-relative frames to the world (anchors are not used past cdof)
      const V3 P = {__shfl(proot.x, B.root), __shfl(proot.y, B.root), __shfl(proot.z, B.root)};
      V3 mxi = {0.f, 0.f, 0.f};
      if (bl && B.b > 0) {
        const V3 xi = v3(S + L.xipos + 3 * B.b) + P;
        mxi = xi * B.mass;
        st3(S + L.xpos + 3 * B.b, v3(S + L.xpos + 3 * B.b) + P);
        st3(S + L.xipos + 3 * B.b, xi);
        st3(S + L.subtree_com + 3 * B.b, v3(S + L.subtree_com + 3 * B.b) + P);
      }
      // the world's subtree spans every tree, each summed in its own frame above: its com
      // again from the world-frame body coms (lane 0 holds the total mass in stm)
      const V3 ms = {wave_sum(mxi.x), wave_sum(mxi.y), wave_sum(mxi.z)};
      if (lane == 0 && stm > MINVAL) st3(S + L.subtree_com, ms * (1.0f / stm));
    }
    sync();
    // site frames: for the sensors and the outputs (and phase C's accelerometers), the last
    // substep's only (nothing in the dynamics reads a site)
    if (last || P->outputs_every) {
      const float* spos = MF(site_pos);
      const float* squat = MF(site_quat);
      for (int s = lane; s < d.nsite; s += kWave) {
        int b = m.site_bodyid[s];
        const Q4 qb = q4(S + L.xquat + 4 * b);
        st3(S + L.sxpos + 3 * s, v3(S + L.xpos + 3 * b) + qrot(qb, v3(spos + 3 * s)));
        qmat(S + L.sxmat + 9 * s, qmul(qb, q4(squat + 4 * s)));
      }
    }
    STAMP(1);
    // =========================================================== CRB + mass matrix
    {
      // composite rigid-body inertia = cinert summed over the subtree (broadcast loop)
      float acc[10];
#pragma unroll
      for (int j = 0; j < 10; j++) acc[j] = 0.f;
#pragma unroll 4
      for (int c = 0; c < nb; c++) {
        const float f = (B.sub >> c) & 1ull ? 1.f : 0.f;
        const float* ci = S + L.cinert + 10 * c;
#pragma unroll
        for (int j = 0; j < 10; j += 2) {
          const float2 v = *reinterpret_cast<const float2*>(ci + j);
          acc[j] = fmaf(f, v.x, acc[j]);
          acc[j + 1] = fmaf(f, v.y, acc[j + 1]);
        }
      }
      if (bl && B.b > 0) {  // the world keeps its (zero) cinert
#pragma unroll
        for (int j = 0; j < 10; j += 2)
          *reinterpret_cast<float2*>(S + L.crb + 10 * B.b + j) = make_float2(acc[j], acc[j + 1]);
      } else if (bl) {
#pragma unroll
        for (int j = 0; j < 10; j++) S[L.crb + j] = S[L.cinert + j];
      }
    }
    sync();
    for (int i = lane; i < nvp * nvp; i += kWave) S[L.M + i] = 0;
    sync();
    for (int i = nv + lane; i < nvp; i += kWave) S[L.M + i * nvp + i] = 1.f;  // identity padding
    if (lane < nv) {
      const int i = lane;
      float f[6];
      inert_mul(f, S + L.crb + 10 * Dr.body, S + L.cdof + 6 * i);
      for (uint64_t a = Dr.anc; a; a &= a - 1) {  // dof i and its ancestors
        const int j = __builtin_ctzll(a);
        float v = dot6(S + L.cdof + 6 * j, f);
        S[L.M + i * nvp + j] = v;
        S[L.M + j * nvp + i] = v;
      }
      S[L.M + i * nvp + i] += Dr.arm;
    }
    sync();
    // M to the B pack now, as its lower tiles (LTR): its LDS slot is reused (in place factor,
    // then contacts).  Phase C gets the implicit-integration factor of M + h D instead
    // (below, scratch region F, also LTR).
    store_ltr(gw + LB.M, S + L.M, nvp, lane);
    STAMP(2);
    // =========================================================== velocity stage
    // cvel(b) = sum over the dofs moving b of cdof * qvel: broadcast loop over the dofs
    {
      float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int j = 0; j < nv; j++) {
        const float f = (B.dofs >> j) & 1ull ? S[L.qvel + j] : 0.f;
        const float* cd = S + L.cdof + 6 * j;
#pragma unroll
        for (int t = 0; t < 6; t += 2) {
          const float2 c2 = *reinterpret_cast<const float2*>(cd + t);
          v[t] = fmaf(f, c2.x, v[t]);
          v[t + 1] = fmaf(f, c2.y, v[t + 1]);
        }
      }
      if (bl) {
#pragma unroll
        for (int t = 0; t < 6; t++) S[L.cvel + 6 * B.b + t] = v[t];
      }
    }
    sync();
    // cdofdot(j) = (velocity before dof j's joint) x cdof(j), mj_comVel: the parent body's
    // cvel plus the earlier joints of the same body; a free joint's rotations see its
    // translations, whose own cdofdot is zero
    if (lane < nv) {
      const int j = lane;
      const bool ftrans = Dr.jt == JNT_FREE && j < Dr.jd0 + 3;
      float v[6];
#pragma unroll
      for (int t = 0; t < 6; t++) v[t] = S[L.cvel + 6 * Dr.pbody + t];
      for (int e = Dr.bd0; e < j; e++) {
        if (e >= Dr.jd0 && !(Dr.jt == JNT_FREE && e < Dr.jd0 + 3)) continue;
        const float q = S[L.qvel + e];
#pragma unroll
        for (int t = 0; t < 6; t++) v[t] += S[L.cdof + 6 * e + t] * q;
      }
      float* cdd = S + L.cdofdot + 6 * j;
      if (ftrans) {
#pragma unroll
        for (int t = 0; t < 6; t++) cdd[t] = 0.f;
      } else {
        cross_motion(cdd, v, S + L.cdof + 6 * j);
      }
    }
    sync();
    // RNE (flg_acc = 0): cacc(b) = -gravity + sum over the dofs moving b of cdofdot * qvel
    // (broadcast loop; handed to phase C as cacc_v), body forces f(b) into the crb slot (dead
    // after M; cdofdot's slot, read by every lane before the barrier), then
    // cfrc(b) = f summed over the subtree into the cacc slot (dead after RNE in phase A)
    {
      float a[6] = {0.f, 0.f, 0.f, -o.gravity[0], -o.gravity[1], -o.gravity[2]};
#pragma unroll 4
      for (int j = 0; j < nv; j++) {
        const float f = (B.dofs >> j) & 1ull ? S[L.qvel + j] : 0.f;
        const float* cd = S + L.cdofdot + 6 * j;
#pragma unroll
        for (int t = 0; t < 6; t += 2) {
          const float2 c2 = *reinterpret_cast<const float2*>(cd + t);
          a[t] = fmaf(f, c2.x, a[t]);
          a[t + 1] = fmaf(f, c2.y, a[t + 1]);
        }
      }
      sync();  // cdofdot (crb slot) read by every lane before the body forces land there
      if (bl) {
        const int b = B.b;
        if (last || P->outputs_every) {  // phase C's post-constraint cacc: the last substep's
#pragma unroll
          for (int t = 0; t < 6; t++) gc[LC.cacc_v + 6 * b + t] = a[t];
        }
        float f1[6], iv[6], f2[6];
        inert_mul(f1, S + L.cinert + 10 * b, a);
        inert_mul(iv, S + L.cinert + 10 * b, S + L.cvel + 6 * b);
        cross_force(f2, S + L.cvel + 6 * b, iv);
        for (int t = 0; t < 6; t++) S[L.crb + 10 * b + t] = f1[t] + f2[t];
      }
    }
    sync();
    {
      float fr[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int c = 0; c < nb; c++) {
        const float f = (B.sub >> c) & 1ull ? 1.f : 0.f;
        const float* fc = S + L.crb + 10 * c;
#pragma unroll
        for (int t = 0; t < 6; t += 2) {
          const float2 c2 = *reinterpret_cast<const float2*>(fc + t);
          fr[t] = fmaf(f, c2.x, fr[t]);
          fr[t + 1] = fmaf(f, c2.y, fr[t + 1]);
        }
      }
      if (bl) {
#pragma unroll
        for (int t = 0; t < 6; t++) S[L.cacc + 6 * B.b + t] = fr[t];
      }
    }
    sync();
    // lane i < nv: qfrc_bias / qfrc_passive of dof i in registers
    float qbias_i = 0.f, qpass_i = 0.f;
    if (lane < nv) {
      const int i = lane;
      qbias_i = dot6(S + L.cdof + 6 * i, S + L.cacc + 6 * Dr.body);  // cfrc
      float pf = -Dr.damp * S[L.qvel + i];
      if ((Dr.jt == JNT_HINGE || Dr.jt == JNT_SLIDE) && Dr.stiff != 0.f)
        pf -= Dr.stiff * (S[L.qpos + Dr.qa] - Dr.qs);
      qpass_i = pf;
    }
    sync();
    // actuation: position / motor actuators on joints.  The actuator forces, qfrc_actuator
    // and qfrc_smooth stay in lane registers (lane u: actuator u, lane i: dof i) and go to
    // the packs from there: no LDS slots (phase A's carve sets its residency)
    float act_f = 0.f, act_gf = 0.f;
    if (lane < nu) {
      const int u = lane;
      const float g = Ar.gear;
      float len = g * S[L.qpos + Ar.qa], vel = g * S[L.qvel + Ar.dof];
      float c = ctrl_u;
      if (Ar.ctrllim) c = fminf(fmaxf(c, Ar.cr0), Ar.cr1);
      float f = Ar.gain * c + Ar.b0 + Ar.b1 * len + Ar.b2 * vel;
      if (Ar.forcelim) f = fminf(fmaxf(f, Ar.fr0), Ar.fr1);
      act_f = f;
      act_gf = g * f;
      if (last) {
        D.actuator_length[(size_t)w * nu + u] = len;
        D.actuator_velocity[(size_t)w * nu + u] = vel;
      }
    }
    // qfrc_actuator of dof i, in lane i: the actuators' g f gathered onto their dofs in
    // actuator order
    float qact_i = 0.f;
    for (int u = 0; u < nu; u++) {
      const float x = rl(act_gf, u);
      if (lane == __builtin_amdgcn_readlane(Ar.dof, u)) qact_i += x;
    }
    float qfs_i = 0.f;  // lane i < nv: qfrc_smooth of dof i
    for (int i = lane; i < nvp; i += kWave) {  // nv <= 64: one pass, lane i
      if (i >= nv) {  // the smooth solve's right-hand side is zero on the padding dofs
        S[L.qacc_smooth + i] = 0.f;
        continue;
      }
      float f = qpass_i - qbias_i + qapp_i + qact_i;
      if (any_xfrc) {
        uint64_t bm = m.dof_bodymask[i];
        const float* cd = S + L.cdof + 6 * i;
        V3 cang = v3(cd), clin = v3(cd + 3);
        for (int b = 1; b < nb; b++) {
          if (!((bm >> b) & 1ull)) continue;
          const float* xf = D.xfrc_applied + ((size_t)w * nb + b) * 6;
          V3 jp = clin + cross(cang, v3(S + L.xipos + 3 * b) - v3(S + L.subtree_com + 3 * m.body_rootid[b]));
          f += dot(jp, v3(xf)) + dot(cang, v3(xf + 3));
        }
      }
      qfs_i = f;
      S[L.qacc_smooth + i] = f;
    }
    if (lane < nvq) {  // both packs (padding zero)
      gw[LB.qfrc_smooth + lane] = qfs_i;
      gc[LC.qfrc_smooth + lane] = qfs_i;
    }
    // subtree momenta (for subtreeangmom sensors and the subtree outputs): like every mjData
    // output of a fused multi-substep step, only the last substep's are observable, so the
    // earlier substeps skip them (and the pos / vel / acc sensors below)
    const bool obs = last != 0 || P->outputs_every;
    if (bl && obs) {
      const int b = B.b;
      const float* cv = S + L.cvel + 6 * b;
      V3 rel = v3(S + L.xipos + 3 * b) - v3(S + L.subtree_com + 3 * B.root);
      V3 vc = v3(cv + 3) + cross(v3(cv), rel);
      st3(S + L.stlin + 3 * b, vc);  // body com velocity; subtree sums below
      float Ri[9];  // ximat
      qmat(Ri, qmul(xq, B.iquat));
      V3 wl = mulTv(Ri, v3(cv));
      V3 hl = {B.inert.x * wl.x, B.inert.y * wl.y, B.inert.z * wl.z};
      st3(S + L.stang + 3 * b, mulv(Ri, hl));
    }
    sync();
    STAMP(6);
    if (integrate) {
      // implicitfast / Euler: factor M + h diag(dof damping - gear^2 biasprm2) here, where M
      // and the (clamped) actuator forces are at hand, into the scratch region F; phase C then
      // runs only the two triangular solves.  The actuator term is dropped for an actuator
      // whose force is at its forcerange limit (zero derivative), as in mj_implicit.
      float act_d = 0.f;
      if (o.integrator == 1 && lane < nu && Ar.b2 != 0.f) {
        bool skip = false;
        if (Ar.forcelim) {
          const float fo = act_f;
          skip = fo <= Ar.fr0 || fo >= Ar.fr1;
        }
        if (!skip) act_d = -h * Ar.gear * Ar.gear * Ar.b2;
      }
      float da = lane < nv ? h * Dr.damp : 0.f;
      for (int u = 0; u < nu; u++) {  // scatter actuator terms onto their dofs
        const float cu = rl(act_d, u);
        if (lane == __builtin_amdgcn_readlane(Ar.dof, u)) da += cu;
      }
      float A[NR];
      float rd;
      if constexpr (kTree<SP>) {  // the factor of the reversed matrix (phase C solves in that order)
        rows_load_rev<NR>(A, S + L.M, nvp, lane);
        const float dp = __shfl(da, lane < nvp ? nvp - 1 - lane : lane);
#pragma unroll
        for (int c = 0; c < NR; c++) A[c] += c == lane ? dp : 0.f;
        rows_chol_tree<NR, SP>(A, rd, S + L.chol, lane);
      } else {
        rows_load<NR>(A, S + L.M, nvp, lane);
#pragma unroll
        for (int c = 0; c < NR; c++) A[c] += c == lane ? da : 0.f;
        rows_chol<NR>(A, rd, S + L.chol, nvp, lane);
      }
      rows_store_strict_ltr<NR>(A, rd, gf, nvp, lane);
    }
    // H <- chol(M); qacc_smooth = M^-1 qfrc_smooth
    if constexpr (kTree<SP>)
      spd_factor_solve_tree<NR, SP>(S + L.M, S + L.H, S + L.qacc_smooth, S + L.chol, nvp, lane);
    else
      spd_factor_solve<NR>(S + L.M, nullptr, S + L.H, S + L.qacc_smooth, S + L.chol, nvp, lane);
    // qacc_smooth to the B pack and a lane register now: its LDS slot (carve.h: dead cinert
    // space) is reused by the geom frames at collision
    const float qacs_i = lane < nvq ? S[L.qacc_smooth + lane] : 0.f;
    if (lane < nvq) gw[LB.qacc_smooth + lane] = qacs_i;
    STAMP(7);
    // subtree com velocity and angular momentum about the subtree com, as sums over the
    // subtree (broadcast loop): V = sum m vc / M, L = sum h + sum m (x - X) x (vc - V) --
    // the closed form of the child-to-parent recursion (parallel-axis shifts)
    if (obs) {
      float* mb = S + L.crb;  // scratch body masses (crb and the RNE forces are dead here)
      if (bl) mb[B.b] = B.mass;
      sync();
      const V3 X = v3(S + L.subtree_com + 3 * B.b);
      const V3 vown = v3(S + L.stlin + 3 * B.b);
      V3 pv = {0.f, 0.f, 0.f}, hs = {0.f, 0.f, 0.f}, cx = {0.f, 0.f, 0.f}, mr = {0.f, 0.f, 0.f};
#pragma unroll 4
      for (int c = 0; c < nb; c++) {
        const bool in = (B.sub >> c) & 1ull;
        const float f = in ? mb[c] : 0.f, fh = in ? 1.f : 0.f;
        const V3 r = v3(S + L.xipos + 3 * c) - X;
        const V3 vc = v3(S + L.stlin + 3 * c);
        pv = pv + vc * f;
        hs = hs + v3(S + L.stang + 3 * c) * fh;
        cx = cx + cross(r, vc) * f;
        mr = mr + r * f;
      }
      sync();  // every lane's reads precede the in-place writes
      if (bl) {
        const float sm = stm;
        const V3 V = sm > MINVAL ? pv * (1.0f / sm) : vown;
        st3(S + L.stlin + 3 * B.b, V);
        st3(S + L.stang + 3 * B.b, hs + cx - cross(mr, V));
      }
      sync();
    }
    // the subtree momenta live in the RNE scratch, which the geom frames take next: their
    // sensors and outputs are written now
    for (int s = lane; obs && s < d.nsensor; s += kWave) {
      if (m.sensor_type[s] != SENS_SUBTREEANGMOM) continue;
      float* out = D.sensordata + (size_t)w * d.nsensordata + m.sensor_adr[s];
      const int obj = m.sensor_objid[s];
      out[0] = S[L.stang + 3 * obj]; out[1] = S[L.stang + 3 * obj + 1]; out[2] = S[L.stang + 3 * obj + 2];
    }
    if (last) {
      const size_t wb = (size_t)w * nb;
      for (int i = lane; i < 3 * nb; i += kWave) {
        D.subtree_linvel[wb * 3 + i] = S[L.stlin + i];
        D.subtree_angmom[wb * 3 + i] = S[L.stang + i];
      }
    }
    sync();
    STAMP(8);
    if (lane == 0) { ints[0] = 0; ints[1] = 0; ints[2] = 0; ints[3] = 0; }
    // geom frames (here, not in kinematics: their LDS aliases regions dead after RNE)
    {
      const float* gpos = MF(geom_pos);
      const float* gquat = MF(geom_quat);
      for (int sl = lane; sl < d.ngeom_lds; sl += kWave) {
        const int g = m.lds_geom[sl];
        int b = m.geom_bodyid[g];
        const Q4 qb = q4(S + L.xquat + 4 * b);
        st3(S + L.gxpos + 3 * sl, v3(S + L.xpos + 3 * b) + qrot(qb, v3(gpos + 3 * g)));
        qmat(S + L.gxmat + 9 * sl, qmul(qb, q4(gquat + 4 * g)));
      }
    }
    sync();
    // =========================================================== collision
    {
      ConOut co{S, ints, &L, d.nconmax};
      const float* gsize = MF(geom_size);
      const float* grb = MF(geom_rbound);
      const float* gmargin = MF(geom_margin);
      // one packed record per pair (capi.cpp pair_rec) while rbound / margin are shared by
      // all worlds; the per-geom load chain otherwise (same values, same fp32 cull radius)
      const bool rec = m.pair_rec != nullptr && m.geom_rbound_ws == 0 && m.geom_margin_ws == 0;
      for (int p = lane; p < d.npair; p += kWave) {
        int g1, g2, t1, t2, l1, l2;  // geoms, types, LDS frame slots
        float margin, cull;
        if (rec) {
          const int4 rc = reinterpret_cast<const int4*>(m.pair_rec)[p];
          g1 = rc.x & 0xffff; g2 = (int)((unsigned)rc.x >> 16);
          l1 = rc.y & 0xfff; l2 = (rc.y >> 12) & 0xfff;
          t1 = (rc.y >> 24) & 15; t2 = (int)((unsigned)rc.y >> 28);
          margin = __int_as_float(rc.z);
          cull = __int_as_float(rc.w);
        } else {
          g1 = m.pair_geom1[p]; g2 = m.pair_geom2[p];
          t1 = m.geom_type[g1]; t2 = m.geom_type[g2];
          l1 = m.geom_lds[g1]; l2 = m.geom_lds[g2];
          margin = fmaxf(gmargin[g1], gmargin[g2]);
          const float r1 = grb[g1], r2 = grb[g2];
          cull = (r1 > 0 && r2 > 0 && t1 != GEOM_HFIELD) ? r1 + r2 + margin : INFINITY;
        }
        V3 p1 = v3(S + L.gxpos + 3 * l1), p2 = v3(S + L.gxpos + 3 * l2);
        if (norm(p2 - p1) > cull) continue;
        const float* s1 = gsize + 3 * g1;
        const float* s2 = gsize + 3 * g2;
        int key = p * 8;
        if (t1 == GEOM_PLANE) {
          const float* Rp = S + L.gxmat + 9 * l1;
          V3 n = {Rp[2], Rp[5], Rp[8]};
          if (t2 == GEOM_SPHERE) {
            plane_sphere(co, key, g1, g2, p1, n, p2, s2[0], margin);
          } else if (t2 == GEOM_CAPSULE) {
            const float* R2 = S + L.gxmat + 9 * l2;
            V3 ax = {R2[2], R2[5], R2[8]};
            int k = key;
            k += plane_sphere(co, k, g1, g2, p1, n, p2 + ax * s2[1], s2[0], margin);
            plane_sphere(co, k, g1, g2, p1, n, p2 - ax * s2[1], s2[0], margin);
          } else if (t2 == GEOM_BOX) {
            float dist = dot(p2 - p1, n);
            const float* R2 = S + L.gxmat + 9 * l2;
            int cnt = 0;
            for (int i = 0; i < 8 && cnt < 4; i++) {
              V3 v = {(i & 1) ? s2[0] : -s2[0], (i & 2) ? s2[1] : -s2[1], (i & 4) ? s2[2] : -s2[2]};
              V3 corner = mulv(R2, v);
              float ld = dot(n, corner);
              if (dist + ld > margin || ld > 0) continue;
              append(co, key + cnt, g1, g2, dist + ld, corner + p2 - n * (0.5f * (dist + ld)), n);
              cnt++;
            }
          } else {
            atomicOr(&ints[3], 4);
          }
        } else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) {
          sphere_sphere(co, key, g1, g2, p1, s1[0], p2, s2[0], margin);
        } else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
          const float* R2 = S + L.gxmat + 9 * l2;
          V3 ax = {R2[2], R2[5], R2[8]};
          V3 pa, pb;
          seg_seg(p1, p1, p2 + ax * s2[1], p2 - ax * s2[1], &pa, &pb);
          sphere_sphere(co, key, g1, g2, p1, s1[0], pb, s2[0], margin);
        } else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
          const float* R1 = S + L.gxmat + 9 * l1;
          const float* R2 = S + L.gxmat + 9 * l2;
          const V3 a1 = {R1[2], R1[5], R1[8]}, a2 = {R2[2], R2[5], R2[8]};
          capsule_capsule(co, key, g1, g2, p1, a1 * s1[1], s1[0], p2, a2 * s2[1], s2[0], margin);
        } else if (t1 == GEOM_BOX && t2 == GEOM_BOX) {
          HFrame F1, F2;
          F1.p = p1; F2.p = p2;
          for (int i = 0; i < 9; i++) { F1.R[i] = S[L.gxmat + 9 * l1 + i]; F2.R[i] = S[L.gxmat + 9 * l2 + i]; }
          if constexpr (kBoxBox<SP>) box_box(co, key, g1, g2, F1, v3(s1), F2, v3(s2), margin);
        } else if (t2 == GEOM_BOX && (t1 == GEOM_SPHERE || t1 == GEOM_CAPSULE)) {
          HFrame F;
          F.p = p2;
#pragma unroll
          for (int i = 0; i < 9; i++) F.R[i] = S[L.gxmat + 9 * l2 + i];
          if (t1 == GEOM_SPHERE) {
            box_sphere(co, key, g1, g2, F, v3(s2), mulTv(F.R, p1 - F.p), s1[0], margin);
          } else {
            const float* R1 = S + L.gxmat + 9 * l1;
            box_capsule(co, key, g1, g2, F, v3(s2), p1, V3{R1[2], R1[5], R1[8]}, s1[1], s1[0], margin);
          }
        } else {
          atomicOr(&ints[3], 4);
        }
      }
      // terrain pairs: chunks of kStaticChunk terrain geoms, then the geoms themselves, are
      // culled by their static world AABBs (capi.cpp) against the union AABB of the partner
      // geoms' bounding spheres; lanes then take the pairs of each overlapping geom.  A
      // terrain of thousands of boxes or hundreds of hfield patches costs ~1-2 chunks and a
      // few geom blocks per world.
      if (d.nstatic > 0) {
        float lo0 = 1e30f, lo1 = 1e30f, lo2 = 1e30f, hi0 = -1e30f, hi1 = -1e30f, hi2 = -1e30f;
        for (int i = lane; i < d.nstpartner; i += kWave) {
          const int g = m.st_partner[i];
          const V3 c = v3(S + L.gxpos + 3 * m.geom_lds[g]);
          const float r = grb[g] + gmargin[g];
          lo0 = fminf(lo0, c.x - r); lo1 = fminf(lo1, c.y - r); lo2 = fminf(lo2, c.z - r);
          hi0 = fmaxf(hi0, c.x + r); hi1 = fmaxf(hi1, c.y + r); hi2 = fmaxf(hi2, c.z + r);
        }
        lo0 = wave_min(lo0); lo1 = wave_min(lo1); lo2 = wave_min(lo2);
        hi0 = wave_max(hi0); hi1 = wave_max(hi1); hi2 = wave_max(hi2);
        auto overlap = [&](const float* bb) {
          return bb[0] <= hi0 && bb[3] >= lo0 && bb[1] <= hi1 && bb[4] >= lo1 && bb[2] <= hi2 &&
                 bb[5] >= lo2;
        };
        const float* gpos = MF(geom_pos);
        const float* gquat = MF(geom_quat);
        const float* hsz_all = MF(hfield_size);
        const float* hdat_all = MF(hfield_data);
        int trunc = 0;
        static_assert(kStaticChunk == kWave, "lane per terrain geom of a chunk");
        const int nchunk = (d.nstatic + kStaticChunk - 1) / kStaticChunk;
        for (int cb = 0; cb < nchunk; cb += kWave) {
          const int c = cb + lane;
          unsigned long long cbal = __ballot(c < nchunk && overlap(m.st_chunk_aabb + 6 * c));
          while (cbal) {
            const int ch = cb + __ffsll((long long)cbal) - 1;
            cbal &= cbal - 1;
            const int i = ch * kStaticChunk + lane;
            unsigned long long bal = __ballot(i < d.nstatic && overlap(m.st_aabb + 6 * i));
            while (bal) {
              const int j = ch * kStaticChunk + __ffsll((long long)bal) - 1;
              bal &= bal - 1;
              const int sg = m.st_geom[j];
              const HFrame F = hfield_frame(m, S, L, gpos, gquat, sg);
              if (m.geom_type[sg] == GEOM_HFIELD) {
                const int hid = m.geom_dataid[sg];
                const float* hs = hsz_all + 4 * hid;
                const float* hd = hdat_all + m.hfield_adr[hid];
                const int nr = m.hfield_nrow[hid], nc = m.hfield_ncol[hid];
                for (int p = m.st_pairadr[j] + lane; p < m.st_pairadr[j + 1]; p += kWave) {
                  const int g2 = m.pair_geom2[p];
                  const int t2 = m.geom_type[g2];
                  const int l2 = m.geom_lds[g2];
                  const V3 p2 = v3(S + L.gxpos + 3 * l2);
                  const float* s2 = gsize + 3 * g2;
                  const float margin = fmaxf(gmargin[sg], gmargin[g2]);
                  const int key = p * 8;
                  if (t2 == GEOM_SPHERE) {
                    hfield_sphere(co, key, sg, g2, F, hd, hs, nr, nc, p2, s2[0], margin, &trunc);
                  } else if (t2 == GEOM_CAPSULE) {
                    const float* R2 = S + L.gxmat + 9 * l2;
                    const V3 ax = {R2[2], R2[5], R2[8]};
                    int k = key;
                    k += hfield_sphere(co, k, sg, g2, F, hd, hs, nr, nc, p2 + ax * s2[1], s2[0], margin, &trunc);
                    hfield_sphere(co, k, sg, g2, F, hd, hs, nr, nc, p2 - ax * s2[1], s2[0], margin, &trunc);
                  } else {
                    atomicOr(&ints[3], 4);
                  }
                }
              } else {  // box welded to the world: its partner is geom 1 (lower geom type),
                        // or either side against another box (geom index order)
                const float* bb = m.st_aabb + 6 * j;
                const V3 bs = v3(gsize + 3 * sg);
                for (int p = m.st_pairadr[j] + lane; p < m.st_pairadr[j + 1]; p += kWave) {
                  const int pa = m.pair_geom1[p], pb = m.pair_geom2[p];
                  const int g1 = pa == sg ? pb : pa;  // the partner
                  const int t1 = m.geom_type[g1];
                  const int l1 = m.geom_lds[g1];
                  const V3 p1 = v3(S + L.gxpos + 3 * l1);
                  const float margin = fmaxf(gmargin[sg], gmargin[g1]);
                  const float rr = grb[g1] + margin;
                  if (p1.x + rr < bb[0] || p1.x - rr > bb[3] || p1.y + rr < bb[1] ||
                      p1.y - rr > bb[4] || p1.z + rr < bb[2] || p1.z - rr > bb[5]) continue;
                  const float* s1 = gsize + 3 * g1;
                  const int key = p * 8;
                  if (t1 == GEOM_SPHERE) {
                    box_sphere(co, key, g1, sg, F, bs, mulTv(F.R, p1 - F.p), s1[0], margin);
                  } else if (t1 == GEOM_CAPSULE) {
                    const float* R1 = S + L.gxmat + 9 * l1;
                    box_capsule(co, key, g1, sg, F, bs, p1, V3{R1[2], R1[5], R1[8]}, s1[1], s1[0], margin);
                  } else if (t1 == GEOM_BOX) {
                    HFrame Fp;
                    Fp.p = p1;
                    for (int i = 0; i < 9; i++) Fp.R[i] = S[L.gxmat + 9 * l1 + i];
                    if constexpr (kBoxBox<SP>) {
                      if (pa == sg) box_box(co, key, pa, pb, F, bs, Fp, v3(s1), margin);
                      else box_box(co, key, pa, pb, Fp, v3(s1), F, bs, margin);
                    }
                  } else {
                    atomicOr(&ints[3], 4);
                  }
                }
              }
            }
          }
        }
        if (trunc) atomicOr(&ints[3], 4);
      }
    }
    sync();
    STAMP(3);
    // deterministic order: bitonic sort of (key, slot) over 64 lanes, then permute (more than
    // 64 contacts: a rank sort, the permutation applied field by field)
    int ncon = min(ints[0], d.nconmax);
    {
      // contact parameters (mj_contactParam semantics) of sorted contact c
      auto contact_params = [&](int c, int g1, int g2, float dist) {
        const float* fri = MF(geom_friction);
        const float* sref = MF(geom_solref);
        const float* simp = MF(geom_solimp);
        const float* smix = MF(geom_solmix);
        const float* gmar = MF(geom_margin);
        const float* ggap = MF(geom_gap);
        int p1 = m.geom_priority[g1], p2 = m.geom_priority[g2];
        int dim;
        float f0, f1;
        float sr[2], si[5];
        if (p1 != p2) {
          int g = p1 > p2 ? g1 : g2;
          dim = m.geom_condim[g];
          f0 = fri[3 * g]; f1 = fri[3 * g + 1];
          sr[0] = sref[2 * g]; sr[1] = sref[2 * g + 1];
          for (int i = 0; i < 5; i++) si[i] = simp[5 * g + i];
        } else {
          dim = max(m.geom_condim[g1], m.geom_condim[g2]);
          f0 = fmaxf(fri[3 * g1], fri[3 * g2]);
          f1 = fmaxf(fri[3 * g1 + 1], fri[3 * g2 + 1]);
          float s1 = smix[g1], s2 = smix[g2], mix;
          if (s1 < MINVAL && s2 < MINVAL) mix = 0.5f;
          else if (s1 < MINVAL) mix = 0.f;
          else if (s2 < MINVAL) mix = 1.f;
          else mix = s1 / (s1 + s2);
          const float* r1 = sref + 2 * g1;
          const float* r2 = sref + 2 * g2;
          if (r1[0] > 0 && r2[0] > 0) {
            sr[0] = mix * r1[0] + (1 - mix) * r2[0];
            sr[1] = mix * r1[1] + (1 - mix) * r2[1];
          } else {
            sr[0] = fminf(r1[0], r2[0]);
            sr[1] = fminf(r1[1], r2[1]);
          }
          for (int i = 0; i < 5; i++) si[i] = mix * simp[5 * g1 + i] + (1 - mix) * simp[5 * g2 + i];
        }
        (void)f1;
        S[L.con_mu + 2 * c] = fmaxf(MINMU, f0);
        S[L.con_mu + 2 * c + 1] = fmaxf(MINMU, f0);
        Si[L.con_dim + c] = dim;
        const float imargin = fmaxf(gmar[g1], gmar[g2]) - fmaxf(ggap[g1], ggap[g2]);
        S[L.con_imargin + c] = imargin;
        // row impedance and reference K, B are per contact: computed once here
        S[L.con_imp + c] = impedance(si, dist, imargin);
        solref_kb(sr, si, h, S[L.con_kb + 2 * c], S[L.con_kb + 2 * c + 1]);
      };
      // con_key is dead after the sort: it then holds the packed contact bodies
      auto con_bodies = [&](int g1, int g2) {
        const int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
        return b1 | b2 << 8 | m.body_rootid[b1] << 16 | m.body_rootid[b2] << 24;
      };
      if (kCon1<SP> || ncon <= kWave) {
        int key = lane < ncon ? Si[L.con_key + lane] : 0x7fffffff;
        int idx = lane;
#pragma unroll
        for (int k = 2; k <= kWave; k <<= 1) {
#pragma unroll
          for (int j = k >> 1; j > 0; j >>= 1) {
            int pk = __shfl_xor(key, j);
            int pi = __shfl_xor(idx, j);
            bool up = (lane & k) == 0;
            bool lower = (lane & j) == 0;
            bool sw = lower ? (up ? key > pk : key < pk) : (up ? key < pk : key > pk);
            if (sw) { key = pk; idx = pi; }
          }
        }
        // lane holds the source slot of sorted position `lane`
        int g1 = 0, g2 = 0;
        float dist = 0, px = 0, py = 0, pz = 0, nx = 0, ny = 0, nz = 0;
        if (lane < ncon) {
          g1 = Si[L.con_g1 + idx]; g2 = Si[L.con_g2 + idx]; dist = S[L.con_dist + idx];
          px = S[L.con_pos + 3 * idx]; py = S[L.con_pos + 3 * idx + 1]; pz = S[L.con_pos + 3 * idx + 2];
          nx = S[L.con_n + 3 * idx]; ny = S[L.con_n + 3 * idx + 1]; nz = S[L.con_n + 3 * idx + 2];
        }
        sync();
        if (lane < ncon) {
          Si[L.con_g1 + lane] = g1; Si[L.con_g2 + lane] = g2; S[L.con_dist + lane] = dist;
          Si[L.con_key + lane] = con_bodies(g1, g2);
          S[L.con_pos + 3 * lane] = px; S[L.con_pos + 3 * lane + 1] = py; S[L.con_pos + 3 * lane + 2] = pz;
          // contact frame (mju_makeFrame): the unit normal; tangents by cframe() at use
          V3 n = {nx, ny, nz};
          n = n * (1.0f / fmaxf(norm(n), MINVAL));
          st3(S + L.con_n + 3 * lane, n);
          contact_params(lane, g1, g2, dist);
        }
      } else if constexpr (!kCon1<SP>) {
        // rank sort (keys pair * 8 + k are distinct): sorted position of slot c = the number
        // of keys below its own; perm[position] = slot in the row-id scratch (rows come later,
        // the carve holds njmax >= nconmax of them)
        int* perm = Si + L.efc_cid;
        const int rounds = (ncon + kWave - 1) / kWave;
        for (int c = lane; c < ncon; c += kWave) {
          const int kc = Si[L.con_key + c];
          int rank = 0;
          for (int j = 0; j < ncon; j++) rank += Si[L.con_key + j] < kc ? 1 : 0;
          perm[rank] = c;
        }
        sync();
        // apply it field by field through registers (at most kMaxConRounds values per lane)
        auto permute = [&](float* base, int stride, int comp) {
          float v[kMaxConRounds];
#pragma unroll
          for (int r = 0; r < kMaxConRounds; r++) {
            const int c = lane + r * kWave;
            v[r] = r < rounds && c < ncon ? base[stride * perm[c] + comp] : 0.f;
          }
          sync();
#pragma unroll
          for (int r = 0; r < kMaxConRounds; r++) {
            const int c = lane + r * kWave;
            if (r < rounds && c < ncon) base[stride * c + comp] = v[r];
          }
          sync();
        };
        permute(reinterpret_cast<float*>(Si + L.con_g1), 1, 0);
        permute(reinterpret_cast<float*>(Si + L.con_g2), 1, 0);
        permute(S + L.con_dist, 1, 0);
        for (int t = 0; t < 3; t++) permute(S + L.con_pos, 3, t);
        for (int t = 0; t < 3; t++) permute(S + L.con_n, 3, t);
        for (int c = lane; c < ncon; c += kWave) {
          const int g1 = Si[L.con_g1 + c], g2 = Si[L.con_g2 + c];
          Si[L.con_key + c] = con_bodies(g1, g2);
          V3 n = v3(S + L.con_n + 3 * c);
          n = n * (1.0f / fmaxf(norm(n), MINVAL));
          st3(S + L.con_n + 3 * c, n);
          contact_params(c, g1, g2, S[L.con_dist + c]);
        }
      }
      sync();
    }
    STAMP(4);
    // =========================================================== constraints
    {
      // row counts: limits (lane per joint) then contacts (lane per contact)
      const float* jrange = MF(jnt_range);
      const float* jmargin = MF(jnt_margin);
      int nlim_rows = 0;
      int lim_mask = 0;  // bit0 lower, bit1 upper
      if (lane < d.njnt && m.jnt_limited[lane] &&
          (m.jnt_type[lane] == JNT_HINGE || m.jnt_type[lane] == JNT_SLIDE)) {
        float q = S[L.qpos + m.jnt_qposadr[lane]];
        float mg = jmargin[lane];
        if (q - jrange[2 * lane] < mg) lim_mask |= 1;
        if (jrange[2 * lane + 1] - q < mg) lim_mask |= 2;
        nlim_rows = (lim_mask & 1) + ((lim_mask >> 1) & 1);
      }
      int lim_total, lim_off = wave_excl_scan(nlim_rows, lane, &lim_total);
      // contact rows: one contact per lane (offsets by one wave scan), or -- past 64 contacts
      // -- rounds of contacts lane + 64 r with a running carry, each contact's offset within
      // the contact rows kept in con_efc (made absolute below)
      const bool con1 = kCon1<SP> || ncon <= kWave;
      int cdim = 0, crow = 0, con_total = 0, con_off = 0;
      if (con1) {
        cdim = lane < ncon ? Si[L.con_dim + lane] : 0;
        crow = lane < ncon ? (cdim == 1 ? 1 : 2 * (cdim - 1)) : 0;
        if (lane < ncon && cdim != 1 && cdim != 3) atomicOr(&ints[3], 4);
        con_off = wave_excl_scan(crow, lane, &con_total);
      } else {
        for (int c0 = 0; c0 < ncon; c0 += kWave) {
          const int c = c0 + lane;
          const int cd = c < ncon ? Si[L.con_dim + c] : 0;
          const int cr = c < ncon ? (cd == 1 ? 1 : 2 * (cd - 1)) : 0;
          if (c < ncon && cd != 1 && cd != 3) atomicOr(&ints[3], 4);
          int tot, off = wave_excl_scan(cr, lane, &tot);
          if (c < ncon) Si[L.con_efc + c] = con_total + off;
          con_total += tot;
        }
      }
      auto con_rows = [&](int c) {
        const int cd = Si[L.con_dim + c];
        return cd == 1 ? 1 : 2 * (cd - 1);
      };
      int nefc = lim_total + con_total;
      if (P->ovf_resolve) {
        // contacts or rows past this carve: list the world for the re-solve at full capacity
        // (the max launch set) instead of dropping whole contacts; a full list falls back to
        // dropping (counted below)
        const bool over = ints[0] > d.nconmax || nefc > d.njmax;
        int slot = -1;
        if (over && lane == 0) {
          const int li = 2 * split + ((sel_arg & kSelAPar) ? 1 : 0);
          slot = atomicAdd(P->ovf_n + li, 1);
          if (slot < P->ovf_cap) {
            P->ovf_list[(size_t)li * P->ovf_cap + slot] = w;
            atomicAdd(D.evtotal + 3, 1);
          }
        }
        slot = __shfl(slot, 0);
        const bool listed = over && slot < P->ovf_cap;
        if (lane == 0) {
          P->ovf_flag[w] = listed ? 1 : 0;
          if (listed) D.nefc[w] = -1;  // classify_kernel leaves the world out
        }
        if (listed) return;
      }
      if (nefc > d.njmax) {
        if (lane == 0) atomicOr(&ints[3], 2);
      }
      // contacts whose rows do not fit are dropped as whole contacts
      int keep_con = ncon;
      if (con1) {
        bool fits = lane < ncon && lim_total + con_off + crow <= d.njmax;
        unsigned long long bal = __ballot(lane < ncon && !fits);
        if (bal) keep_con = __ffsll((long long)bal) - 1;
        keep_con = min(keep_con, ncon);
        ncon = keep_con;
        nefc = lim_total + (ncon > 0 ? __shfl(con_off + crow, ncon - 1) : 0);
      } else {
        for (int c0 = 0; c0 < ncon; c0 += kWave) {
          const int c = c0 + lane;
          const bool fits = c < ncon && lim_total + Si[L.con_efc + c] + con_rows(c) <= d.njmax;
          const unsigned long long bal = __ballot(c < ncon && !fits);
          if (bal) { keep_con = c0 + __ffsll((long long)bal) - 1; break; }
        }
        ncon = keep_con;
        nefc = lim_total + (ncon > 0 ? Si[L.con_efc + ncon - 1] + con_rows(ncon - 1) : 0);
      }
      if (lim_total > d.njmax) { nefc = 0; ncon = 0; }
      const float* dinvw = MF(dof_invweight0);
      const float* binvw = MF(body_invweight0);
      const float* jsolref = MF(jnt_solref);
      const float* jsolimp = MF(jnt_solimp);
      // limit rows metadata (J set below) -- lane per joint
      if (lim_mask && nefc > 0) {
        int r = lim_off;
        float q = S[L.qpos + m.jnt_qposadr[lane]];
        for (int side = -1; side <= 1; side += 2) {
          if (!((side < 0 ? lim_mask & 1 : lim_mask & 2))) continue;
          float dist = side * (jrange[2 * lane + (side + 1) / 2] - q);
          Si[L.efc_cid + r] = efc_code(EFC_LIMIT, lane | m.jnt_dofadr[lane] << 8);
          S[L.efc_aref + r] = dist;       // temporarily: pos
          S[L.efc_D + r] = (float)(-side);  // temporarily: jacobian sign
          r++;
        }
      }
      // ints[6]: some contact couples two branches of the dof tree (neither body's dofs
      // contain the other's), so its rows fill the Newton Hessian outside the tree pattern
      // and phase B factors it densely; otherwise the tree form (rows_chol_tree)
      bool xbranch = false;
      if constexpr (kTree<SP>) {
        for (int c = lane; c < ncon; c += kWave) {
          const int cbk = Si[L.con_key + c];
          const uint64_t m1 = m.body_dofmask[cb_b1(cbk)], m2 = m.body_dofmask[cb_b2(cbk)];
          xbranch |= (m1 & ~m2) != 0ull && (m2 & ~m1) != 0ull;
        }
      }
      const int dense_h = __ballot(xbranch) != 0ull || !kTree<SP>;
      if (con1) {
        if (lane < ncon) {
          int r0 = lim_total + con_off;
          Si[L.con_efc + lane] = r0;
          for (int k = 0; k < crow; k++)
            Si[L.efc_cid + r0 + k] = efc_code(cdim == 1 ? EFC_FRICTIONLESS : EFC_PYRAMIDAL, lane);
        }
      } else {
        for (int c = lane; c < ncon; c += kWave) {
          const int r0 = lim_total + Si[L.con_efc + c];
          const int cd = Si[L.con_dim + c];
          Si[L.con_efc + c] = r0;
          for (int k = 0; k < con_rows(c); k++)
            Si[L.efc_cid + r0 + k] = efc_code(cd == 1 ? EFC_FRICTIONLESS : EFC_PYRAMIDAL, c);
        }
      }
      sync();
      // Jacobian rows: lane per dof; when nvp <= 32 the wave holds kWave / nvp groups of nvp
      // lanes that take every ngrp-th row / contact (Go1, nvp 20: 3 contacts at once instead
      // of 20 active lanes of 64)
      const int ngrp = nvp <= kWave / 2 ? kWave / nvp : 1;
      const int grp = lane / nvp;
      for (int i = lane - grp * nvp; grp < ngrp && i < nvp; i += kWave) {
        // limits
        for (int r = grp; r < lim_total && r < nefc; r += ngrp) {
          const int jd = Si[L.efc_cid + r] >> 2;
          Jg[r * nvp + i] = (jd >> 8) == i ? S[L.efc_D + r] : 0.f;
        }
        if (i >= nv) {  // zero padding columns of the contact rows
          for (int r = lim_total + grp; r < nefc; r += ngrp) Jg[r * nvp + i] = 0.f;
          continue;
        }
        uint64_t bm = m.dof_bodymask[i];
        const float* cd = S + L.cdof + 6 * i;
        V3 cang = v3(cd), clin = v3(cd + 3);
        for (int c = grp; c < ncon; c += ngrp) {
          const int cb = Si[L.con_key + c];
          const int b1 = cb_b1(cb), b2 = cb_b2(cb);
          V3 pos = v3(S + L.con_pos + 3 * c);
          V3 jd = {0, 0, 0};
          if (b2 > 0 && ((bm >> b2) & 1ull))
            jd = jd + clin + cross(cang, pos - v3(S + L.subtree_com + 3 * cb_r2(cb)));
          if (b1 > 0 && ((bm >> b1) & 1ull))
            jd = jd - (clin + cross(cang, pos - v3(S + L.subtree_com + 3 * cb_r1(cb))));
          const CFrame F = cframe(v3(S + L.con_n + 3 * c));
          float jn = dot(F.n, jd);
          int r0 = Si[L.con_efc + c];
          if (Si[L.con_dim + c] == 1) {
            Jg[r0 * nvp + i] = jn;
          } else {
            float jt1 = dot(F.t, jd);
            float jt2 = dot(F.b, jd);
            float mu0 = S[L.con_mu + 2 * c], mu1 = S[L.con_mu + 2 * c + 1];
            Jg[(r0 + 0) * nvp + i] = jn + mu0 * jt1;
            Jg[(r0 + 1) * nvp + i] = jn - mu0 * jt1;
            Jg[(r0 + 2) * nvp + i] = jn + mu1 * jt2;
            Jg[(r0 + 3) * nvp + i] = jn - mu1 * jt2;
          }
        }
      }
      sync();
      // row parameters: lane per row
      for (int r = lane; r < nefc; r += kWave) {
        const int code = Si[L.efc_cid + r];
        const int type = code & 3, pl = code >> 2;  // pl: contact, or joint | dof << 8
        float pos, margin, diag, imp, K, B;
        if (type == EFC_LIMIT) {
          const int j = pl & 255;
          pos = S[L.efc_aref + r];
          margin = jmargin[j];
          diag = dinvw[pl >> 8];
          imp = impedance(jsolimp + 5 * j, pos, margin);
          solref_kb(jsolref + 2 * j, jsolimp + 5 * j, h, K, B);
        } else {
          const int c = pl;
          pos = S[L.con_dist + c];
          margin = S[L.con_imargin + c];
          const int cb = Si[L.con_key + c];
          float tran = binvw[2 * cb_b1(cb)] + binvw[2 * cb_b2(cb)];
          if (type == EFC_FRICTIONLESS) {
            diag = tran;
          } else {
            float mu = S[L.con_mu + 2 * c + ((r - Si[L.con_efc + c]) >> 1)];
            diag = (tran + mu * mu * tran) / o.impratio;
          }
          imp = S[L.con_imp + c];
          K = S[L.con_kb + 2 * c];
          B = S[L.con_kb + 2 * c + 1];
        }
        float Rr = fmaxf(MINVAL, (1 - imp) * diag / imp);
        // efc_vel = J qvel, evaluated from the body velocities (cvel is the same chain sum)
        float vel;
        if (type == EFC_LIMIT) {
          vel = S[L.efc_D + r] * S[L.qvel + (pl >> 8)];
        } else {
          const int c = pl;
          V3 pc = v3(S + L.con_pos + 3 * c);
          const int cb = Si[L.con_key + c];
          V3 v = point_vel_r(S, L, cb_b2(cb), cb_r2(cb), pc) - point_vel_r(S, L, cb_b1(cb), cb_r1(cb), pc);
          const CFrame F = cframe(v3(S + L.con_n + 3 * c));
          vel = dot(F.n, v);
          if (type != EFC_FRICTIONLESS) {
            int kr = r - Si[L.con_efc + c];
            const V3 t = (kr >> 1) ? F.b : F.t;
            float mu = S[L.con_mu + 2 * c + (kr >> 1)];
            vel += ((kr & 1) ? -mu : mu) * dot(t, v);
          }
        }
        S[L.efc_D + r] = 1.0f / Rr;
        S[L.efc_aref + r] = -B * vel - K * imp * (pos - margin);
      }
      if (lane == 0) { ints[1] = nefc; ints[2] = lim_total; ints[4] = ncon; ints[6] = dense_h; }
      sync();
    }
    const int nefc = ints[1];
    ncon = ints[4];
    if (lane == 0) D.nefc[w] = nefc;  // every substep: classify_kernel sorts the Newton work by it
    STAMP(5);
    // =========================================================== sensors
    // (pos / vel stage: the last substep's only, see the subtree momenta above)
    for (int s = lane; obs && s < d.nsensor; s += kWave) {
      float* out = D.sensordata + (size_t)w * d.nsensordata + m.sensor_adr[s];
      int obj = m.sensor_objid[s];
      int type = m.sensor_type[s];
      // pos/vel-stage sensors run in phase A, acceleration-stage ones in phase C
      if ((type == SENS_ACCELEROMETER || type == SENS_CONTACT) != (PH == 2)) continue;
      // single-slot contact sensors: wave-cooperative below (contact_sensors_wave), unless
      // there are more than 64 of them (no transposed masks) or more than 64 contacts
      if (type == SENS_CONTACT && m.sensor_intprm[3 * s + 2] <= 1 && m.ncsens > 0 &&
          (kCon1<SP> || ncon <= kWave)) continue;
      if (type == SENS_GYRO || type == SENS_VELOCIMETER || type == SENS_ACCELEROMETER) {
        int b = m.site_bodyid[obj];
        const float* R = S + L.sxmat + 9 * obj;
        const float* cv = S + L.cvel + 6 * b;
        V3 rel = v3(S + L.sxpos + 3 * obj) - v3(S + L.subtree_com + 3 * m.body_rootid[b]);
        V3 r;
        if (type == SENS_GYRO) {
          r = mulTv(R, v3(cv));
        } else {
          V3 v = v3(cv + 3) + cross(v3(cv), rel);
          if (type == SENS_VELOCIMETER) {
            r = mulTv(R, v);
          } else {
            const float* ca = S + L.cacc + 6 * b;
            V3 a = v3(ca + 3) + cross(v3(ca), rel) + cross(v3(cv), v);
            r = mulTv(R, a);
          }
        }
        out[0] = r.x; out[1] = r.y; out[2] = r.z;
      } else if (type == SENS_SUBTREEANGMOM) {
        // written right after the subtree momenta (phase A; their LDS is reused since)
      } else if (type == SENS_FRAMEPOS) {
        const float* p = m.sensor_objtype[s] == OBJ_SITE ? S + L.sxpos + 3 * obj : S + L.xpos + 3 * obj;
        out[0] = p[0]; out[1] = p[1]; out[2] = p[2];
      } else if (type == SENS_JOINTPOS) {
        out[0] = S[L.qpos + m.jnt_qposadr[obj]];
      } else if (type == SENS_JOINTVEL) {
        out[0] = S[L.qvel + m.jnt_dofadr[obj]];
      } else if (type == SENS_CONTACT) {
        const int32_t* ip = m.sensor_intprm + 3 * s;
        int bits = ip[0], reduce = ip[1], nslot = min(ip[2], 8);
        const uint32_t* mk1 = m.sensor_geommask1 + m.nmaskword * s;
        const uint32_t* mk2 = m.sensor_geommask2 + m.nmaskword * s;
        int fdim = ((bits & 1) || (bits & 8)) ? 1 : 3;
        int dim = m.sensor_dim[s];
        for (int i = 0; i < dim; i++) out[i] = 0.f;
        int found = 0;
        V3 net = {0, 0, 0};
        int sel[8];
        float key[8];
        int nsel = 0;
        for (int c = 0; c < ncon; c++) {
          int g1 = Si[L.con_g1 + c], g2 = Si[L.con_g2 + c];
          bool a1 = ((mk1[g1 >> 5] >> (g1 & 31)) & 1u) && ((mk2[g2 >> 5] >> (g2 & 31)) & 1u);
          bool a2 = ((mk1[g2 >> 5] >> (g2 & 31)) & 1u) && ((mk2[g1 >> 5] >> (g1 & 31)) & 1u);
          if (!a1 && !a2) continue;
          if (found >= o.maxmatch) continue;  // contact_sensor_maxmatch: the first matches only
          found++;
          // contact force in contact frame
          int r0 = Si[L.con_efc + c];
          V3 f = {0, 0, 0};
          if (Si[L.con_dim + c] == 1) {
            f.x = S[L.efc_force + r0];
          } else {
            float e0 = S[L.efc_force + r0], e1 = S[L.efc_force + r0 + 1];
            float e2 = S[L.efc_force + r0 + 2], e3 = S[L.efc_force + r0 + 3];
            f = {e0 + e1 + e2 + e3, (e0 - e1) * S[L.con_mu + 2 * c], (e2 - e3) * S[L.con_mu + 2 * c + 1]};
          }
          V3 fg = frame_tv(S + L.con_n + 3 * c, f);
          net = net + fg * (a1 ? 1.f : -1.f);
          float k = reduce == REDUCE_MINDIST ? S[L.con_dist + c]
                  : reduce == REDUCE_MAXFORCE ? -norm(f) : (float)nsel;
          if (nsel < nslot || k < key[nsel - 1]) {
            int pos = nsel < nslot ? nsel++ : nslot - 1;
            while (pos > 0 && key[pos - 1] > k) { key[pos] = key[pos - 1]; sel[pos] = sel[pos - 1]; pos--; }
            key[pos] = k;
            sel[pos] = c * 2 + (a1 ? 0 : 1);
          }
        }
        if (reduce == REDUCE_NETFORCE) {
          if (bits & 1) out[0] = (float)found;
          else if (bits & 2) { out[0] = net.x; out[1] = net.y; out[2] = net.z; }
        } else {
          for (int k = 0; k < nsel; k++) {
            int c = sel[k] >> 1;
            float sg = (sel[k] & 1) ? -1.f : 1.f;
            float* oo = out + k * fdim;
            if (bits & 1) oo[0] = (float)found;
            else if (bits & 8) oo[0] = S[L.con_dist + c];
            else if (bits & 16) { for (int t = 0; t < 3; t++) oo[t] = S[L.con_pos + 3 * c + t]; }
            else if (bits & 32) { for (int t = 0; t < 3; t++) oo[t] = sg * S[L.con_n + 3 * c + t]; }
            else if (bits & 64) { for (int t = 0; t < 3; t++) oo[t] = sg * vc(cframe(v3(S + L.con_n + 3 * c)).t, t); }
            else if (bits & 2) {
              int r0 = Si[L.con_efc + c];
              if (Si[L.con_dim + c] == 1) { oo[0] = S[L.efc_force + r0]; oo[1] = oo[2] = 0; }
              else {
                float e0 = S[L.efc_force + r0], e1 = S[L.efc_force + r0 + 1];
                float e2 = S[L.efc_force + r0 + 2], e3 = S[L.efc_force + r0 + 3];
                oo[0] = e0 + e1 + e2 + e3;
                oo[1] = (e0 - e1) * S[L.con_mu + 2 * c];
                oo[2] = (e2 - e3) * S[L.con_mu + 2 * c + 1];
              }
            }
          }
        }
      }
    }
    STAMP(11);
    // outputs final after phase A
#ifdef MJX_ABLATE_OUTPUTS
    if (false) {
#else
    if (last) {
#endif
      size_t wb = (size_t)w * nb;
      for (int i = lane; i < 3 * nb; i += kWave) {
        D.xpos[wb * 3 + i] = S[L.xpos + i];
        D.xipos[wb * 3 + i] = S[L.xipos + i];
        D.subtree_com[wb * 3 + i] = S[L.subtree_com + i];
      }
      for (int i = lane; i < 4 * nb; i += kWave) D.xquat[wb * 4 + i] = S[L.xquat + i];
      if (bl) {  // lane per body: xmat and ximat from the quaternions
        float R[9], Ri[9];
        qmat(R, xq);
        qmat(Ri, qmul(xq, B.iquat));
        float* om = D.xmat + (wb + B.b) * 9;
        float* oi = D.ximat + (wb + B.b) * 9;
#pragma unroll
        for (int t = 0; t < 9; t++) { om[t] = R[t]; oi[t] = Ri[t]; }
      }
      for (int i = lane; i < 6 * nb; i += kWave) D.cvel[wb * 6 + i] = S[L.cvel + i];
      // lane per geom: one model-index load per lane up front, not one per element (a
      // dependent global load in every iteration of an element loop serialises on latency);
      // heightfield frames are static (set at sim creation)
      size_t wg = (size_t)w * d.ngeom;
      for (int i = lane; i < d.ngeom_lds; i += kWave) {
        const size_t g = wg + m.lds_geom[i];
        const float* xp = S + L.gxpos + 3 * i;
        const float* xm = S + L.gxmat + 9 * i;
        float* op = D.geom_xpos + g * 3;
        float* om = D.geom_xmat + g * 9;
#pragma unroll
        for (int t = 0; t < 3; t++) op[t] = xp[t];
#pragma unroll
        for (int t = 0; t < 9; t++) om[t] = xm[t];
      }
      size_t ws = (size_t)w * d.nsite;
      for (int i = lane; i < 3 * d.nsite; i += kWave) D.site_xpos[ws * 3 + i] = S[L.sxpos + i];
      for (int i = lane; i < 9 * d.nsite; i += kWave) D.site_xmat[ws * 9 + i] = S[L.sxmat + i];
      for (int i = lane; i < nv; i += kWave) {
        size_t k = (size_t)w * nv + i;
        D.qacc_smooth[k] = qacs_i;  // lane i (nv <= 64)
        D.qfrc_bias[k] = qbias_i;
        D.qfrc_passive[k] = qpass_i;
        D.qfrc_actuator[k] = qact_i;
        D.qfrc_smooth[k] = qfs_i;
      }
      if (lane < nu) D.actuator_force[(size_t)w * nu + lane] = act_f;
      size_t wc = (size_t)w * P->con_stride;
      // contact slots: this output's contacts, and zeros over the previous output's past them
      // (every slot beyond both is zero already: engine_counters [6] = slots this output
      // touches, [7] = contacts it holds)
      int* wsv = D.wstats + 8 * (size_t)w;
      const int nout = min(P->con_stride, max(ncon, wsv[7]));
      for (int c = lane; c < nout; c += kWave) {
        bool v = c < ncon;
        D.contact_dist[wc + c] = v ? S[L.con_dist + c] : 0.f;
        D.contact_geom[(wc + c) * 2] = v ? Si[L.con_g1 + c] : -1;
        D.contact_geom[(wc + c) * 2 + 1] = v ? Si[L.con_g2 + c] : -1;
        for (int t = 0; t < 3; t++) D.contact_pos[(wc + c) * 3 + t] = v ? S[L.con_pos + 3 * c + t] : 0.f;
        const CFrame F = cframe(v ? v3(S + L.con_n + 3 * c) : V3{0.f, 0.f, 1.f});
        const float fr[9] = {F.n.x, F.n.y, F.n.z, F.t.x, F.t.y, F.t.z, F.b.x, F.b.y, F.b.z};
        for (int t = 0; t < 9; t++) D.contact_frame[(wc + c) * 9 + t] = v ? fr[t] : 0.f;
      }
      if (lane == 0) { D.ncon[w] = ncon; D.nefc[w] = nefc; wsv[6] = nout; wsv[7] = ncon; }
    }
    STAMP(12);
    // hand-off: B pack (J rows already written) and the A part of the C pack; the contact
    // arrays only up to the live contacts (phase C reads none past ncon)
    const int C = ncon;
    const int C4 = (C + 3) & ~3;
    const int nr4 = (nefc + 3) & ~3;
    cp4(gw + LB.ints, S + L.ints, 8, lane);  // (qacc_smooth, qfrc_smooth: stored above)
    cp4(gw + LB.efc_aref, S + L.efc_aref, nr4, lane);
    cp4(gw + LB.efc_D, S + L.efc_D, nr4, lane);
    // (the C pack's last-substep part only in the last substep: carve.h packC)
    if (obs) {
      cp4(gc + LC.cdof, S + L.cdof, 6 * nvp, lane);
      cp4(gc + LC.cvel, S + L.cvel, (6 * nb + 3) & ~3, lane);
      cp4(gc + LC.subtree_com, S + L.subtree_com, (3 * nb + 3) & ~3, lane);
    }
    if (obs) {
      cp4(gc + LC.sxpos, S + L.sxpos, (3 * d.nsite + 3) & ~3, lane);
      cp4(gc + LC.sxmat, S + L.sxmat, (9 * d.nsite + 3) & ~3, lane);
    }
    cp4(gc + LC.con_g1, S + L.con_g1, C4, lane);
    cp4(gc + LC.con_g2, S + L.con_g2, C4, lane);
    if (obs) {
      cp4(gc + LC.con_dist, S + L.con_dist, C4, lane);
      cp4(gc + LC.con_pos, S + L.con_pos, (3 * C + 3) & ~3, lane);
      cp4(gc + LC.con_n, S + L.con_n, (3 * C + 3) & ~3, lane);  // normals (C rebuilds frames)
      cp4(gc + LC.con_mu, S + L.con_mu, (2 * C + 3) & ~3, lane);
      cp4(gc + LC.con_dim, S + L.con_dim, C4, lane);
      cp4(gc + LC.con_efc, S + L.con_efc, C4, lane);
    }
    STAMP(14);
  } else if constexpr (PH == 1) {
    // ----------------------------------------------------------- phase B (Newton)
    {
      const int nefc_in = reinterpret_cast<const int*>(gw)[LB.ints + 1];
      // row classes (launch_step, classify_kernel): class k > 0 holds the worlds with
      // row_cap[k-2] < nefc <= row_cap[k-1], class 0 the rest (all worlds without classes)
      const int cls = integrate;
      // B pack: carve offsets == pack offsets; M's slot holds M in LTR form (the rest of the
      // slot is neither written nor read)
      cp_pack(S, gw, L.M + ltr_size(nvp), lane);
      if (JG) {
        // the pack up to J (its offsets equal this carve's); J stays in global memory
        cp_pack(S + L.qacc_smooth, gw + LB.qacc_smooth, LB.efc_J - LB.qacc_smooth, lane);
      } else if (cls <= 0) {
        cp_pack(S + L.qacc_smooth, gw + L.qacc_smooth, L.efc_J + nefc_in * nvp - L.qacc_smooth, lane);
      } else {
        // the pack is laid out with the full-capacity carve LB: [ints M qacc_smooth
        // qfrc_smooth efc_aref] sit at the same offsets in both, efc_D and efc_J move
        const int nr4 = (nefc_in + 3) & ~3;
        cp_pack(S + L.qacc_smooth, gw + LB.qacc_smooth, LB.efc_aref + nr4 - LB.qacc_smooth, lane);
        cp_pack(S + L.efc_D, gw + LB.efc_D, nr4, lane);
        cp_pack(S + L.efc_J, gw + LB.efc_J, nefc_in * nvp, lane);
      }
    }
    const Tiles T = make_tiles(nvp, lane);
    for (int i = lane; i < nvp; i += kWave) {
      S[L.x + i] = 0.f; S[L.Mx + i] = 0.f;
      S[L.srch + i] = 0.f; S[L.Ms + i] = 0.f; S[L.qfrc_con + i] = 0.f;
      S[L.qacc_ws + i] = i < nv ? D.qacc_warmstart[(size_t)w * nv + i] : 0.f;
    }
    lds_dma_wait();
    sync();
    const int nefc = ints[1];
    int ncon = ints[4];
    (void)ncon;
    // tree-pattern Hessian (no contact across two branches of the dof tree, phase A's
    // ints[6]): factored in the fill-free reversed order, rows_chol_tree
    const bool tree_h = kTree<SP> && !MJX_JTDJ_MFMA && __builtin_amdgcn_readfirstlane(ints[6]) == 0;
    float Mt[2][16];  // M as register tiles; its LDS slot becomes H / jt_mul scratch
    tiles_load_ltr(Mt, T, S + L.M);
    sync();
    STAMP(15);
    // =========================================================== Newton solver
    int niter = 0;
    if (nefc == 0) {
      for (int i = lane; i < nvp; i += kWave) {
        S[L.x + i] = S[L.qacc_smooth + i];
        S[L.qfrc_con + i] = 0.f;
      }
      sync();
    } else {
      float* jar = S + L.efc_jar;
      float* Js = S + L.efc_Js;
      float* wv = S + L.efc_force;
      const float* Dv = S + L.efc_D;
      // (JG: the B pack's rows in global memory, written by this world's phase A in an earlier
      // launch -- a kernel boundary, so no stale vector-L1 line)
      const float* J = JG ? gw + LB.efc_J : S + L.efc_J;
      int* act = Si + L.efc_act;
      float* Lm = S + L.H;
      const float scale = 1.0f / (o.meaninertia * (float)max(nv, 1));
#ifdef MJX_STAMPS
      sub_prev = __builtin_amdgcn_s_memtime();
      stamp_acc[38] += 1;         // solves with rows
      stamp_acc[39] += !tree_h;   // of them with the dense factor (a contact across branches)
#endif
      // With at most one row per lane (every world of the bulk row class) the solver keeps
      // its row's D, J x - aref (rja) and, in the line search, J s (rjs) in registers: the
      // per-row loops below then read no LDS.  Lanes past nefc hold zeros (v = 0 is never
      // active), so every sum is the loop form's, bit for bit; jar stays mirrored in LDS.
      const bool reg_rows = nefc <= kWave;
      const float rD = reg_rows && lane < nefc ? Dv[lane] : 0.f;
      float rja = 0.f;
      // jar = J x - aref for every row (lane per row)
      auto set_jar = [&](const float* xv) {
        matvec_rows(jar, J, xv, nefc, nvp, lane);
        for (int r = lane; r < nefc; r += kWave) jar[r] -= S[L.efc_aref + r];
        if (reg_rows) rja = lane < nefc ? jar[lane] : 0.f;
      };
      // total cost at (x, Mx, jar): Gauss term + active half-quadratics (wave-uniform)
      auto cost_of = [&](const float* xv, const float* Mxv) -> float {
        float g = 0.f;
        for (int i = lane; i < nv; i += kWave)
          g += 0.5f * (xv[i] - S[L.qacc_smooth + i]) * (Mxv[i] - S[L.qfrc_smooth + i]);
        if (reg_rows) {
          if (rja < 0.f) g += 0.5f * rD * rja * rja;
        } else {
          for (int r = lane; r < nefc; r += kWave) {
            float v = jar[r];
            if (v < 0.f) g += 0.5f * Dv[r] * v * v;
          }
        }
        return wave_sum(g);
      };
      // lane i's dof values in registers for the iterations (nvp <= 64): x, M x (mirrored
      // in LDS, which the J x products and the output copies read) and the constant
      // qacc_smooth / qfrc_smooth; same per-lane arithmetic as the LDS loops
      float rx = 0.f, rMx = 0.f, rqs = 0.f, rfs = 0.f;
      auto cost_now = [&]() -> float {
        float g = 0.f;
        if (lane < nv) g += 0.5f * (rx - rqs) * (rMx - rfs);
        if (reg_rows) {
          if (rja < 0.f) g += 0.5f * rD * rja * rja;
        } else {
          for (int r = lane; r < nefc; r += kWave) {
            float v = jar[r];
            if (v < 0.f) g += 0.5f * Dv[r] * v * v;
          }
        }
        return wave_sum(g);
      };
      // warmstart: keep qacc_warmstart if its cost beats qacc_smooth
      for (int i = lane; i < nvp; i += kWave) S[L.x + i] = S[L.qacc_ws + i];
      sync();
      tiles_symv(Mt, T, S + L.x, S + L.Mx, nvp, lane);
      set_jar(S + L.x);
      sync();
      const float cost_ws = cost_of(S + L.x, S + L.Mx);
      sync();
      set_jar(S + L.qacc_smooth);
      sync();
      const float cost_sm = cost_of(S + L.qacc_smooth, S + L.qfrc_smooth);
      sync();
      float cost;
      if (cost_sm < cost_ws) {
        for (int i = lane; i < nvp; i += kWave) {
          S[L.x + i] = S[L.qacc_smooth + i];
          S[L.Mx + i] = S[L.qfrc_smooth + i];
        }
        cost = cost_sm;
      } else {
        set_jar(S + L.x);
        cost = cost_ws;
      }
      sync();
      if (lane < nvp) {
        rx = S[L.x + lane];
        rMx = S[L.Mx + lane];
        rqs = S[L.qacc_smooth + lane];
        rfs = S[L.qfrc_smooth + lane];
      }
      SUBSTAMP(0);
      unsigned long long act_sig[4] = {~0ull, ~0ull, ~0ull, ~0ull};
      for (int iter = 0; iter < o.iterations; iter++) {
        // gradient = M x - qfrc_smooth + J_act^T (D jar)
        bool same_set;
        int nchg = 0;
        const int nact = reg_rows ? build_active1(act, rja, nefc, lane, act_sig, &same_set, &nchg)
                                  : build_active(act, jar, nefc, lane, act_sig, &same_set, &nchg);
        // H depends on the active set only: unchanged set -> reuse the stored factor (exact)
        const bool refactor = iter == 0 || !same_set;
#ifdef MJX_STAMPS
        stamp_acc[40] += 1;
        stamp_acc[41] += refactor && iter > 0;
        stamp_acc[42] += iter > 0 ? nchg : 0;
        stamp_acc[43] += refactor && iter > 0 && nchg <= 4;
        stamp_acc[44] += iter == 0 ? nact : 0;
#endif
        (void)nchg;
        if (reg_rows) {
          if (lane < nefc) wv[lane] = rD * rja;
        } else {
          for (int r = lane; r < nefc; r += kWave) wv[r] = Dv[r] * jar[r];
        }
        sync();
        jt_mul(S + L.srch, J, wv, act, nact, nvp, lane);
        float gn = 0.f, gr = 0.f;
        if (lane < nvp) {
          const int i = lane;
          const float jf = S[L.srch + i], mx = rMx, fs = rfs;
          const float g = jf + mx - fs;  // gradient
          S[L.srch + i] = -g;
          gn += g * g;
          const float a = fabsf(jf) + fabsf(mx) + fabsf(fs);
          gr += a * a;
        }
        gn = sqrtf(wave_sum(gn));
        gr = sqrtf(wave_sum(gr));
        SUBSTAMP(1);
        // MuJoCo's gradient test; floor = fp32 rounding scale of the summed terms
        if (iter > 0 && scale * gn < fmaxf(o.tolerance, 16.f * FLT_EPSILON * scale * gr)) break;
        // Hessian H = M + J_act^T D J_act in register tiles, factor, solve
        if (refactor) {
#if MJX_JTDJ_MFMA
          tiles_store(Mt, T, Lm, nvp);
          sync();
          mfma_add_jtdj<NR>(Lm, J, Dv, act, nact, nvp, lane);
#else
          float A[2][16];
#pragma unroll
          for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
            for (int e2 = 0; e2 < 16; e2++) A[s2][e2] = Mt[s2][e2];
          tiles_add_jtdj(A, T, J, Dv, act, nact, nvp);
          if (tree_h) tiles_store_rev_ltr(A, T, Lm);  // H in LTR form (carve.h, phase B)
          else tiles_store_ltr(A, T, Lm);
#endif
        }
        sync();
        SUBSTAMP(2);
        {
          float R[NR];
          float rd;
          if (refactor) {
#if MJX_JTDJ_MFMA
            rows_load<NR>(R, Lm, nvp, lane);
            rows_chol<NR, (LAT & 1) != 0>(R, rd, S + LB.chol, nvp, lane);
            rows_store_strict<NR>(R, rd, Lm, nvp, lane);
#else
            rows_load_ltr<NR>(R, Lm, nvp, lane);  // the reversed matrix's rows when tree_h
            if (tree_h) {
              if constexpr (kTree<SP>) rows_chol_tree<NR, SP>(R, rd, S + LB.chol, lane);
            } else {
              rows_chol<NR, (LAT & 1) != 0>(R, rd, S + LB.chol, nvp, lane);  // M / chol offsets are the same in every row-class carve
            }
            rows_store_strict_ltr<NR>(R, rd, Lm, nvp, lane);
#endif
            rows_fwd_rows<NR>(R, rd, lane);
          } else {
#if MJX_JTDJ_MFMA
            rows_load_factor<NR>(R, rd, Lm, nvp, lane);
#else
            rows_load_factor_ltr<NR>(R, rd, Lm, nvp, lane);
#endif
          }
          sync();
          SUBSTAMP(3);
          // the tree-form factor is of the reversed matrix: lane i solves for dof nvp-1-i
          const int pl = tree_h ? nvp - 1 - lane : lane;
          float xs = lane < nvp ? S[L.srch + pl] : 0.f;
#if MJX_JTDJ_MFMA
          xs = rows_solve<NR>(R, rd, Lm, xs, nvp, lane);
#else
          xs = rows_solve_ltr<NR>(R, rd, Lm, xs, nvp, lane);
#endif
          sync();
          if (lane < nvp) S[L.srch + pl] = xs;
          sync();
        }
        SUBSTAMP(4);
        matvec_rows(Js, J, S + L.srch, nefc, nvp, lane);
        tiles_symv(Mt, T, S + L.srch, S + L.Ms, nvp, lane);
        float g1 = 0.f, sn = 0.f, sv = 0.f;
        if (lane < nv) {
          sv = S[L.srch + lane];
          g1 += sv * (rMx - rfs);
          sn += sv * sv;
        }
        sync();
        float g2 = 0.f;
        if (lane < nv) g2 += sv * S[L.Ms + lane];
        g1 = wave_sum(g1);
        g2 = wave_sum(g2);
        sn = sqrtf(wave_sum(sn));
        const float gtol = o.tolerance * o.ls_tolerance * sn / scale;
        // the line search's J s (constant across its evaluations) in a register too
        const float rjs = reg_rows && lane < nefc ? Js[lane] : 0.f;
        SUBSTAMP(5);
        // exact line search on the piecewise-quadratic cost (same algorithm as the oracle)
        // The derivative is a sum of O(nefc) terms; once |der| is within its fp32
        // rounding floor the root of the piecewise-linear derivative has been found to
        // working precision (gtol itself, 1e-10 relative by default, is an fp64 target).
        auto ls_eval = [&](float alpha, float* der, float* der2, float* noise) {
          float f1 = 0.f, f2 = 0.f, fa = 0.f;
          if (reg_rows) {
            const float v = rja + alpha * rjs;
            if (v < 0) {
              const float t = rD * v * rjs;
              f1 += t;
              fa += fabsf(t);
              f2 += rD * rjs * rjs;
            }
          } else {
            for (int r = lane; r < nefc; r += kWave) {
              float js = Js[r];
              float v = jar[r] + alpha * js;
              if (v < 0) {
                float Dr = Dv[r];
                float t = Dr * v * js;
                f1 += t;
                fa += fabsf(t);
                f2 += Dr * js * js;
              }
            }
          }
          f1 = wave_sum(f1);
          f2 = wave_sum(f2);
          fa = wave_sum(fa);
          *der = g1 + alpha * g2 + f1;
          *der2 = g2 + f2;
          *noise = 64.f * FLT_EPSILON * (fabsf(g1) + fabsf(alpha * g2) + fa);
        };
        float d0, dd0, nz0;
        ls_eval(0.f, &d0, &dd0, &nz0);
        float alpha = 0.f;
        if (d0 < 0) {
          float c0 = 0.f;
          if (reg_rows) {
            if (rja < 0 || (rja == 0 && rjs < 0)) c0 += rD * rjs * rjs;
          } else {
            for (int r = lane; r < nefc; r += kWave) {
              float ja = jar[r], js = Js[r];
              if (ja < 0 || (ja == 0 && js < 0)) c0 += Dv[r] * js * js;
            }
          }
          c0 = g2 + wave_sum(c0);
          float lo = 0.f, hi = -1.f, best = 0.f;
          float a = -d0 / c0;
          bool done = false;
          for (int it = 0; it < o.ls_iterations; it++) {
            float der, der2, nz;
#ifdef MJX_STAMPS
            stamp_acc[45] += 1;
#endif
            ls_eval(a, &der, &der2, &nz);
            if (fabsf(der) <= fmaxf(gtol, nz)) { alpha = a; done = true; break; }
            if (der < 0) { lo = a; best = a; } else { hi = a; }
            float next = der2 > 0 ? a - der / der2 : a * 2;
            if (hi >= 0 && !(next > lo && next < hi)) next = 0.5f * (lo + hi);
            if (hi < 0 && next <= lo) next = lo + (lo > 0 ? lo : 1.0f);
            a = next;
          }
          if (!done) alpha = best > 0 ? best : a;
#ifdef MJX_STAMPS
          stamp_acc[46] += 1;
#endif
        }
        niter = iter + 1;
        SUBSTAMP(6);
        if (alpha == 0.f) break;
        if (lane < nvp) {
          rx = rx + alpha * S[L.srch + lane];
          rMx = rMx + alpha * S[L.Ms + lane];
          S[L.x + lane] = rx;
          S[L.Mx + lane] = rMx;
        }
        if (reg_rows) {
          rja = rja + alpha * rjs;  // lanes past nefc: 0 + alpha * 0
          if (lane < nefc) jar[lane] = rja;
        } else {
          for (int r = lane; r < nefc; r += kWave) jar[r] += alpha * Js[r];
        }
        sync();
        float old = cost;
        cost = cost_now();
        SUBSTAMP(7);
        // MuJoCo's improvement test, with the fp32 resolution of the cost (a sum of
        // non-negative terms, so its rounding error is ~eps*|cost|) as the floor: below
        // it, further iterations only chase rounding noise.
        if (scale * (old - cost) < fmaxf(o.tolerance, 4.f * FLT_EPSILON * scale * fabsf(cost))) break;
      }
      // constraint forces and qfrc_constraint = J^T f over the active rows
      sync();
      if (reg_rows) {
        if (lane < nefc) wv[lane] = rja < 0 ? -rD * rja : 0.f;
      } else {
        for (int r = lane; r < nefc; r += kWave) {
          float ja = jar[r];
          wv[r] = ja < 0 ? -Dv[r] * ja : 0.f;
        }
      }
      unsigned long long sig_f[4] = {0, 0, 0, 0};
      bool same_f;
      const int nact = reg_rows ? build_active1(act, rja, nefc, lane, sig_f, &same_f)
                                : build_active(act, jar, nefc, lane, sig_f, &same_f);
      sync();
      jt_mul(S + L.qfrc_con, J, wv, act, nact, nvp, lane);
      SUBSTAMP(8);
    }
    STAMP(9);
    if (lane == 0) ints[5] = niter;
    sync();
    cp4(gc + LC.ints, S + L.ints, 8, lane);
    cp4(gc + LC.x, S + L.x, nvq, lane);
    cp4(gc + LC.qfrc_con, S + L.qfrc_con, nvq, lane);
    if (last || P->outputs_every)  // phase C reads the row forces in the last substep only
      cp4(gc + LC.efc_force, S + L.efc_force, (nefc + 3) & ~3, lane);
    if (last) {
      for (int i = lane; i < nv; i += kWave) {
        size_t k = (size_t)w * nv + i;
        D.qacc[k] = S[L.x + i];
        D.qfrc_constraint[k] = S[L.qfrc_con + i];
      }
      if (lane == 0) D.solver_niter[w] = niter;
    }
    STAMP(14);
  } else {
    // ----------------------------------------------------------- phase C
    // C pack (carve offsets == pack offsets): before the last substep of a fused step only
    // the part every substep reads and phase B's ints / qacc / qfrc_constraint (carve.h)
    if (last || P->outputs_every) {
      cp_pack(S, gc, L.pack_len, lane);
    } else {
      cp_pack(S, gc, L.packC_sub, lane);
      cp_pack(S + L.ints, gc + L.ints, L.efc_force - L.ints, lane);
    }
    // the implicit-integration factor (phase A stored it): in flight with the pack
    float Fa[NR], Fdv = 1.f;
    if (integrate) rows_load_factor_ltr_raw<NR>(Fa, Fdv, gf, nvp, lane);
    for (int i = lane; i < nvp; i += kWave) {
      const bool in = i < nv;
      S[L.qvel + i] = in ? D.qvel[(size_t)w * nv + i] : 0.f;
      S[L.qacc_ws + i] = in ? D.qacc_warmstart[(size_t)w * nv + i] : 0.f;
    }
    for (int i = lane; i < nq; i += kWave) S[L.qpos + i] = D.qpos[(size_t)w * nq + i];
    float time = D.time[w];
    const BodyLite B = load_body_lite(m, d, min(lane, nb - 1));
    const bool bl = lane < nb;
    lds_dma_wait();
    sync();
    const int nefc = ints[1];
    int ncon = ints[4];
    const int niter_last = ints[5];
    STAMP(15);
    // =========================================================== post-constraint acc
    // cacc(b) = cacc_v(b) + sum over the dofs moving b of cdof * qacc, cacc_v(b) = -gravity
    // + sum cdofdot * qvel from phase A's RNE (broadcast loop over the dofs, no level syncs);
    // for the accelerometers and the cacc output: the last substep's only
    if (last || P->outputs_every) {
      float a[6];
#pragma unroll
      for (int t = 0; t < 6; t++) a[t] = S[L.cacc_v + 6 * B.b + t];
#pragma unroll 4
      for (int j = 0; j < nv; j++) {
        const float fa = (B.dofs >> j) & 1ull ? S[L.x + j] : 0.f;
        const float* cd = S + L.cdof + 6 * j;
#pragma unroll
        for (int t = 0; t < 6; t += 2) {
          const float2 c2 = *reinterpret_cast<const float2*>(cd + t);
          a[t] = fmaf(fa, c2.x, a[t]);
          a[t + 1] = fmaf(fa, c2.y, a[t + 1]);
        }
      }
      if (bl) {
#pragma unroll
        for (int t = 0; t < 6; t++) S[L.cacc + 6 * B.b + t] = a[t];
      }
    }
    sync();
    STAMP(10);
    // =========================================================== sensors
    for (int s = lane; s < d.nsensor; s += kWave) {
      float* out = D.sensordata + (size_t)w * d.nsensordata + m.sensor_adr[s];
      int obj = m.sensor_objid[s];
      int type = m.sensor_type[s];
      // pos/vel-stage sensors run in phase A, acceleration-stage ones in phase C
      if ((type == SENS_ACCELEROMETER || type == SENS_CONTACT) != (PH == 2)) continue;
      // the accelerometers: the last substep's only (contact sensors run every substep: the
      // contact air times read their found counts)
      if (!last && !P->outputs_every) {
        if (type != SENS_CONTACT) continue;
        bool air = false;  // a contact sensor whose found count a contact air time reads
        for (int i = 0; i < P->nair; i++) air |= P->air_found[i] == m.sensor_adr[s];
        if (!air) continue;
      }
      // single-slot contact sensors: wave-cooperative below (contact_sensors_wave), unless
      // there are more than 64 of them (no transposed masks)
      if (type == SENS_CONTACT && m.sensor_intprm[3 * s + 2] <= 1 && m.ncsens > 0 &&
          (kCon1<SP> || ncon <= kWave)) continue;
      if (type == SENS_GYRO || type == SENS_VELOCIMETER || type == SENS_ACCELEROMETER) {
        int b = m.site_bodyid[obj];
        const float* R = S + L.sxmat + 9 * obj;
        const float* cv = S + L.cvel + 6 * b;
        V3 rel = v3(S + L.sxpos + 3 * obj) - v3(S + L.subtree_com + 3 * m.body_rootid[b]);
        V3 r;
        if (type == SENS_GYRO) {
          r = mulTv(R, v3(cv));
        } else {
          V3 v = v3(cv + 3) + cross(v3(cv), rel);
          if (type == SENS_VELOCIMETER) {
            r = mulTv(R, v);
          } else {
            const float* ca = S + L.cacc + 6 * b;
            V3 a = v3(ca + 3) + cross(v3(ca), rel) + cross(v3(cv), v);
            r = mulTv(R, a);
          }
        }
        out[0] = r.x; out[1] = r.y; out[2] = r.z;
      } else if (type == SENS_SUBTREEANGMOM) {
        // written right after the subtree momenta (phase A; their LDS is reused since)
      } else if (type == SENS_FRAMEPOS) {
        const float* p = m.sensor_objtype[s] == OBJ_SITE ? S + L.sxpos + 3 * obj : S + L.xpos + 3 * obj;
        out[0] = p[0]; out[1] = p[1]; out[2] = p[2];
      } else if (type == SENS_JOINTPOS) {
        out[0] = S[L.qpos + m.jnt_qposadr[obj]];
      } else if (type == SENS_JOINTVEL) {
        out[0] = S[L.qvel + m.jnt_dofadr[obj]];
      } else if (type == SENS_CONTACT) {
        const int32_t* ip = m.sensor_intprm + 3 * s;
        int bits = ip[0], reduce = ip[1], nslot = min(ip[2], 8);
        const uint32_t* mk1 = m.sensor_geommask1 + m.nmaskword * s;
        const uint32_t* mk2 = m.sensor_geommask2 + m.nmaskword * s;
        int fdim = ((bits & 1) || (bits & 8)) ? 1 : 3;
        int dim = m.sensor_dim[s];
        for (int i = 0; i < dim; i++) out[i] = 0.f;
        int found = 0;
        V3 net = {0, 0, 0};
        int sel[8];
        float key[8];
        int nsel = 0;
        for (int c = 0; c < ncon; c++) {
          int g1 = Si[L.con_g1 + c], g2 = Si[L.con_g2 + c];
          bool a1 = ((mk1[g1 >> 5] >> (g1 & 31)) & 1u) && ((mk2[g2 >> 5] >> (g2 & 31)) & 1u);
          bool a2 = ((mk1[g2 >> 5] >> (g2 & 31)) & 1u) && ((mk2[g1 >> 5] >> (g1 & 31)) & 1u);
          if (!a1 && !a2) continue;
          if (found >= o.maxmatch) continue;  // contact_sensor_maxmatch: the first matches only
          found++;
          // contact force in contact frame
          int r0 = Si[L.con_efc + c];
          V3 f = {0, 0, 0};
          if (Si[L.con_dim + c] == 1) {
            f.x = S[L.efc_force + r0];
          } else {
            float e0 = S[L.efc_force + r0], e1 = S[L.efc_force + r0 + 1];
            float e2 = S[L.efc_force + r0 + 2], e3 = S[L.efc_force + r0 + 3];
            f = {e0 + e1 + e2 + e3, (e0 - e1) * S[L.con_mu + 2 * c], (e2 - e3) * S[L.con_mu + 2 * c + 1]};
          }
          V3 fg = frame_tv(S + L.con_n + 3 * c, f);
          net = net + fg * (a1 ? 1.f : -1.f);
          float k = reduce == REDUCE_MINDIST ? S[L.con_dist + c]
                  : reduce == REDUCE_MAXFORCE ? -norm(f) : (float)nsel;
          if (nsel < nslot || k < key[nsel - 1]) {
            int pos = nsel < nslot ? nsel++ : nslot - 1;
            while (pos > 0 && key[pos - 1] > k) { key[pos] = key[pos - 1]; sel[pos] = sel[pos - 1]; pos--; }
            key[pos] = k;
            sel[pos] = c * 2 + (a1 ? 0 : 1);
          }
        }
        if (reduce == REDUCE_NETFORCE) {
          if (bits & 1) out[0] = (float)found;
          else if (bits & 2) { out[0] = net.x; out[1] = net.y; out[2] = net.z; }
        } else {
          for (int k = 0; k < nsel; k++) {
            int c = sel[k] >> 1;
            float sg = (sel[k] & 1) ? -1.f : 1.f;
            float* oo = out + k * fdim;
            if (bits & 1) oo[0] = (float)found;
            else if (bits & 8) oo[0] = S[L.con_dist + c];
            else if (bits & 16) { for (int t = 0; t < 3; t++) oo[t] = S[L.con_pos + 3 * c + t]; }
            else if (bits & 32) { for (int t = 0; t < 3; t++) oo[t] = sg * S[L.con_n + 3 * c + t]; }
            else if (bits & 64) { for (int t = 0; t < 3; t++) oo[t] = sg * vc(cframe(v3(S + L.con_n + 3 * c)).t, t); }
            else if (bits & 2) {
              int r0 = Si[L.con_efc + c];
              if (Si[L.con_dim + c] == 1) { oo[0] = S[L.efc_force + r0]; oo[1] = oo[2] = 0; }
              else {
                float e0 = S[L.efc_force + r0], e1 = S[L.efc_force + r0 + 1];
                float e2 = S[L.efc_force + r0 + 2], e3 = S[L.efc_force + r0 + 3];
                oo[0] = e0 + e1 + e2 + e3;
                oo[1] = (e0 - e1) * S[L.con_mu + 2 * c];
                oo[2] = (e2 - e3) * S[L.con_mu + 2 * c + 1];
              }
            }
          }
        }
      }
    }
    if (kCon1<SP> || ncon <= kWave)
      contact_sensors_wave(S, Si, L, m, d, D.sensordata + (size_t)w * d.nsensordata, ncon,
                           o.maxmatch, last || P->outputs_every, P, lane);
    STAMP(11);
    if (last) {
      size_t wb = (size_t)w * nb;
      for (int i = lane; i < 6 * nb; i += kWave) D.cacc[wb * 6 + i] = S[L.cacc + i];
      size_t wc = (size_t)w * P->con_stride;
      const int nout = min(P->con_stride, D.wstats[8 * (size_t)w + 6]);  // phase A's output slots
      for (int c = lane; c < nout; c += kWave) {
        V3 f = {0, 0, 0};
        if (c < ncon && nefc > 0) {
          int r0 = Si[L.con_efc + c];
          if (Si[L.con_dim + c] == 1) f.x = S[L.efc_force + r0];
          else {
            float e0 = S[L.efc_force + r0], e1 = S[L.efc_force + r0 + 1];
            float e2 = S[L.efc_force + r0 + 2], e3 = S[L.efc_force + r0 + 3];
            f = {e0 + e1 + e2 + e3, (e0 - e1) * S[L.con_mu + 2 * c], (e2 - e3) * S[L.con_mu + 2 * c + 1]};
          }
        }
        D.contact_force[(wc + c) * 3] = f.x;
        D.contact_force[(wc + c) * 3 + 1] = f.y;
        D.contact_force[(wc + c) * 3 + 2] = f.z;
      }
    }
    // per-world counters, every substep (a fused multi-substep step must not lose the
    // overflow events of its earlier substeps): [0,1,5] running max, [2..4] event counts
    if (lane < 6) {
      int* ws = D.wstats + 8 * (size_t)w;
      const int v = lane == 0 ? ints[0] : lane == 1 ? nefc : lane == 5 ? niter_last
                  : (ints[3] >> (lane - 2)) & 1;
      const int old = ws[lane];
      ws[lane] = (lane >= 2 && lane <= 4) ? old + v : max(old, v);
      if (lane >= 2 && lane <= 4 && v) atomicAdd(D.evtotal + lane - 2, v);
    }
    STAMP(12);
#ifdef MJX_STAMPS
    sub_prev = __builtin_amdgcn_s_memtime();
#endif
    if (integrate) {
      sync();
    // =========================================================== implicitfast / Euler
    sync();
    {
      SUBSTAMP(9);
      // (M + h D) qacc' = qfrc_smooth + qfrc_constraint with the factor phase A stored in
      // the world's scratch (rows and columns come straight from global memory)
      SUBSTAMP(10);
      {
        float rd;
        rows_scale_factor_ltr<NR>(Fa, rd, Fdv, nvp, lane);
        // a tree-form factor (phase A) is of the reversed matrix: lane i solves for dof nvp-1-i
        const int pl = kTree<SP> ? nvp - 1 - lane : lane;
        const float f = lane < nvp ? S[L.qfrc_smooth + pl] + S[L.qfrc_con + pl] : 0.f;
        const float acc = rows_solve_ltr<NR>(Fa, rd, gf, f, nvp, lane);
        if (lane < nvp && pl < nv) S[L.qvel + pl] += h * acc;
      }
      sync();
      SUBSTAMP(11);
      for (int k = lane; k < d.njnt; k += kWave) {
        int a = m.jnt_qposadr[k], dof = m.jnt_dofadr[k];
        int t = m.jnt_type[k];
        if (t == JNT_FREE) {
          for (int i = 0; i < 3; i++) S[L.qpos + a + i] += h * S[L.qvel + dof + i];
          V3 wv = v3(S + L.qvel + dof + 3);
          float nw = norm(wv);
          V3 ax = nw < MINVAL ? V3{1, 0, 0} : wv * (1.0f / nw);
          Q4 q = qnorm(q4(S + L.qpos + a + 3));
          q = qmul(q, qaxisangle(ax, h * nw));
          st4(S + L.qpos + a + 3, q);
        } else if (t == JNT_HINGE || t == JNT_SLIDE) {
          S[L.qpos + a] += h * S[L.qvel + dof];
        }
      }
      for (int i = lane; i < nv; i += kWave) S[L.qacc_ws + i] = S[L.x + i];
      time += h;
      sync();
      SUBSTAMP(12);
    }

      for (int i = lane; i < nq; i += kWave) D.qpos[(size_t)w * nq + i] = S[L.qpos + i];
      for (int i = lane; i < nv; i += kWave) {
        D.qvel[(size_t)w * nv + i] = S[L.qvel + i];
        D.qacc_warmstart[(size_t)w * nv + i] = S[L.qacc_ws + i];
      }
      if (lane == 0) D.time[w] = time;
      // contact-sensor air time (ContactSensor._update_air_time_tracking,
      // sensor/contact_sensor.py:327-367): the found values this phase stored above are
      // read back after a workgroup fence (other lanes wrote them)
      const int nair = P->nair;
      if (nair > 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const float el = time - P->air_time[w];
        if (lane < nair) {
          const size_t i = (size_t)w * nair + lane;
          const bool contact = D.sensordata[(size_t)w * d.nsensordata + P->air_found[lane]] > 0.f;
          const float ca = P->air_cur[i], cc = P->air_cc[i];
          if (ca > 0.f && contact) P->air_last[i] = ca + el;
          P->air_cur[i] = contact ? 0.f : ca + el;
          if (cc > 0.f && !contact) P->air_lc[i] = cc + el;
          P->air_cc[i] = contact ? cc + el : 0.f;
        }
        if (lane == 0) P->air_time[w] = time;
      }
    }
    STAMP(13);
  }
  STAMP_FLUSH();
#ifdef MJX_STAMPS
  if (lane == 0) {
    D.wtrace[(size_t)w * 8 + 2 * PH] = wt0;
    D.wtrace[(size_t)w * 8 + 2 * PH + 1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// An overflow re-solve launch (step_ovf) has a fixed grid (kOvfGrid, captured in graphs);
// each workgroup takes listed worlds bid, bid + grid, ... until the list's count.  Every
// other launch runs one world per workgroup.
__device__ __forceinline__ bool ovf_more(const Params* __restrict__ P, int sel, int bid) {
  if (!(sel & kSelOvf)) return false;
  const int li = 2 * (sel & 0xff) + ((sel & kSelRPar) ? 1 : 0);
  if (bid >= min(P->ovf_n[li], P->ovf_cap)) return false;
  __syncthreads();  // the wave's LDS carve is reused by the next world
  return true;
}

template <int NR, int PH, int SP>
__global__ __launch_bounds__(kWave) MJX_PHASE_ATTR void step_phase(const Params* __restrict__ P, int w0, int w1,
                                                    int sel, int last, int integrate,
                                                    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  step_body<NR, PH, SP, false>(S, P, w0, w1, sel, last, integrate, mask, (int)blockIdx.x);
}
// Phase B for the full-capacity row class (the heavy worlds: more constraint rows than the
// class capacity) and the masked forward.  That launch holds a few hundred worlds on 256 CUs,
// one wave per SIMD at most, so its span is one world's latency, not throughput: the kernel
// may take 256 VGPRs (2 waves / SIMD, still above its LDS-bound residency) and spends them
// on loads issued ahead of their use (rows_chol<NR, true>).
// JGL = 3: the constraint Jacobian read from the B pack in global memory (carve kLdsJG): the
// heavy worlds' full-capacity carve shrinks by njmax x nvp floats, so they hold a fraction of
// the LDS the concurrent bulk class needs, and more of them fit a CU where they are many.
// CAP: the same code at the throughput kernels' register budget (3 waves / SIMD), so that a
// SIMD running a heavy world keeps two bulk-class waves beside it instead of one
template <int NR, int SP, int JGL = 1, int CAP = 0>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(CAP ? 3 : 1, CAP ? 8 : 2))) void step_newton_lat(
    const Params* __restrict__ P, int w0, int w1, int sel, int last, int integrate,
    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  step_body<NR, 1, SP, JGL>(S, P, w0, w1, sel, last, integrate, mask, (int)blockIdx.x);
}
// The full-capacity class's Newton in the throughput form (3 waves / SIMD) with J in global
// memory: for batches whose heavy worlds are many (jump hfield: ~5,400 of 16,384 at 84-137
// rows), where that launch is throughput-bound, not one world's latency.
template <int NR, int SP>
__global__ __launch_bounds__(kWave) MJX_PHASE_ATTR_B void step_phase_jg(
    const Params* __restrict__ P, int w0, int w1, int sel, int last, int integrate,
    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  step_body<NR, 1, SP, 2>(S, P, w0, w1, sel, last, integrate, mask, (int)blockIdx.x);
}

// The overflow re-solve launches (sel & kSelOvf; ovf_chain): a fixed grid of kOvfGrid
// workgroups, each looping over the listed worlds.  A separate entry, so that the loop's
// live ranges stay out of the bulk kernels (inlined into step_phase the loop cost phase A 74
// VGPRs and phase C 64); its few worlds need no residency.
// The launch flagged kSelClr is the list's last reader: its last workgroup out empties the
// list (count and done counter) for the substep after next -- no launch of its own.
// An empty list (the common case: nothing overflowed the fast carve) was read by nobody and
// needs no clearing: its workgroups skip the agent-scope fence, whose L2 write-back made each
// near-empty launch cost ~15 us (in line on the critical path of split batches, Go1 8,192).
__device__ __forceinline__ void ovf_clear_on_exit(const Params* __restrict__ P, int sel) {
  if (!(sel & kSelClr)) return;
  const int li = 2 * (sel & 0xff) + ((sel & kSelRPar) ? 1 : 0);
  if (threadIdx.x == 0) {
    // (the count is fixed for the whole launch: only its last workgroup out clears it)
    if (P->ovf_n[li] == 0) return;
    __threadfence();  // this workgroup's reads of the list precede the count
    if (atomicAdd(P->ovf_done + li, 1) == (int)gridDim.x - 1) {
      P->ovf_n[li] = 0;
      P->ovf_done[li] = 0;
    }
  }
}

template <int NR, int PH, int SP, int LAT>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(1, 2))) void step_ovf(
    const Params* __restrict__ P, int w0, int w1, int sel, int last, int integrate,
    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  for (int bid = (int)blockIdx.x;; bid += (int)gridDim.x) {
    step_body<NR, PH, SP, LAT>(S, P, w0, w1, sel, last, integrate, mask, bid);
    if (!ovf_more(P, sel, bid + (int)gridDim.x)) break;
  }
  ovf_clear_on_exit(P, sel);
}

// The re-solve of a listed world's whole substep in the max carve as ONE launch (phase A,
// the latency Newton kernel, phase C back to back per world, hand-offs through the max
// scratch): an empty list then costs one near-empty launch per substep instead of three.
// LDS: the largest of the three carves.
template <int NR, int SP>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(1, 1))) void step_resolve(
    const Params* __restrict__ P, int w0, int w1, int sel, int last, int integrate,
    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  if (sel & kSelOvf) {  // a workgroup past the listed count: no world, no fences
    const int li = 2 * (sel & 0xff) + ((sel & kSelRPar) ? 1 : 0);
    if ((int)blockIdx.x >= min(P->ovf_n[li], P->ovf_cap)) {
      ovf_clear_on_exit(P, sel);
      return;
    }
  }
  for (int bid = (int)blockIdx.x;; bid += (int)gridDim.x) {
    step_body<NR, 0, SP, false>(S, P, w0, w1, sel, last, integrate, mask, bid);
    __threadfence();  // the packs this wave stored are read back by the next phase
    __syncthreads();
    step_body<NR, 1, SP, true>(S, P, w0, w1, sel, last, -1, mask, bid);
    __threadfence();
    __syncthreads();
    step_body<NR, 2, SP, false>(S, P, w0, w1, sel, last, integrate, mask, bid);
    if (!ovf_more(P, sel, bid + (int)gridDim.x)) break;
  }
  ovf_clear_on_exit(P, sel);
}

// A row class's chain as ONE launch (MJX355_CHAIN, engine.hip class_chain): per world its
// Newton (the class's carve; LAT: the latency form for the full-capacity class), its phase C
// and -- kSelChainA -- the next substep's phase A, back to back in the workgroup, the packs
// handed over through the per-world scratch as between launches.  A world then flows through
// B -> C -> A on its own: the launch boundaries no longer make every world of the class wait
// for the class's slowest Newton (7-10 iterations against a median of 3) before its phase C,
// and for the slowest phase C before its next phase A.  sel: split | (class + 1) << 8 |
// kSelChainA | kSelAPar (next A's list parity) | kSelNextLast; `integrate` as for phase C.
// Between phases: a workgroup-scope release (this wave's pack stores complete before the
// next phase's LDS-DMA reads them; one wave per workgroup, same CU) -- not an agent-scope
// fence, whose L2 write-back cost the earlier fused C + A launch 24 %.
__device__ __forceinline__ void chain_handoff() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
template <int NR, int SP, int LAT>
__global__ __launch_bounds__(kWave)
__attribute__((amdgpu_waves_per_eu((LAT & 1) ? 1 : (kLean<SP> ? 4 : NR <= 48 ? 3 : 1), (LAT & 1) ? 2 : 8))) void step_chain(
    const Params* __restrict__ P, int w0, int w1, int sel, int last, int integrate,
    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  const int bid = (int)blockIdx.x;
  const int split = sel & 0xff;
  const int cls1 = (sel >> 8) & 0xff;  // class + 1
  step_body<NR, 1, SP, LAT>(S, P, w0, w1, split, last, cls1 - 1, mask, bid);
  chain_handoff();
  step_body<NR, 2, SP, 0>(S, P, w0, w1, split | cls1 << 8, last, integrate, mask, bid);
  if (sel & kSelChainA) {
    chain_handoff();
    step_body<NR, 0, SP, 0>(S, P, w0, w1, split | cls1 << 8 | (sel & kSelAPar) | kSelFusedA,
                                (sel & kSelNextLast) ? 1 : 0, integrate, mask, bid);
  }
}

// The masked forward (the reset worlds of an env step) in the max carve as ONE launch: phase
// A, the latency Newton kernel and phase C back to back per masked world, hand-offs as in
// step_chain.  A workgroup whose world is not masked exits at once.  LDS: the largest of the
// three max carves.  (Three launches cost two more dispatch ramps and launch gaps on the env
// step's critical path, for the handful of worlds a step resets.)
template <int NR, int SP>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(1, 2))) void step_masked(
    const Params* __restrict__ P, int w0, int w1, int sel, int last, int integrate,
    const uint8_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) float S[];
  const int bid = (int)blockIdx.x;
  if (w0 + bid >= w1 || !mask[w0 + bid]) return;
  step_body<NR, 0, SP, false>(S, P, w0, w1, sel, last, integrate, mask, bid);
  chain_handoff();
  step_body<NR, 1, SP, true>(S, P, w0, w1, sel, last, -1, mask, bid);
  chain_handoff();
  step_body<NR, 2, SP, false>(S, P, w0, w1, sel, last, integrate, mask, bid);
}

using StepFn = void (*)(const Params*, int, int, int, int, int, const uint8_t*);

// kernel of phase code ph: 0 A, 1 B, 2 C, 3 B latency form; 4: phase A over a re-solve list
// (the fast carve's next substep), 5: a listed world's whole substep (step_resolve); 6 / 7: a
// row class's B -> C -> next A chain as one launch (step_chain; 7: the latency form); 8: the
// masked forward's A -> B -> C in the max carve (step_masked)
template <int NR, int SP>
StepFn phase_kernel(int ph) {
  constexpr int role = SpecRole<SP>::mask;
  switch (ph) {
    case 0: return step_phase<NR, 0, SP>;
    case 2: return step_phase<NR, 2, SP>;
    case 3: return step_newton_lat<NR, SP>;
    case 4:
      if constexpr ((role & 1) != 0) return step_ovf<NR, 0, SP, false>;
      else return nullptr;
    case 1:
      if constexpr ((role & 1) != 0) return step_phase<NR, 1, SP>;
      else return nullptr;
    case 5:
      if constexpr ((role & 2) != 0) return step_resolve<NR, SP>;
      else return nullptr;
    case 6:
      if constexpr ((role & 1) != 0) return step_chain<NR, SP, false>;
      else return nullptr;
    case 7:
      if constexpr ((role & 1) != 0) return step_chain<NR, SP, true>;
      else return nullptr;
    case 8:
      if constexpr ((role & 2) != 0) return step_masked<NR, SP>;
      else return nullptr;
    case 9:
      if constexpr ((role & 1) != 0) return step_newton_lat<NR, SP, 3>;
      else return nullptr;
    case 10:  // the full-capacity class's Newton, throughput form, J in global memory
      if constexpr ((role & 1) != 0) return step_phase_jg<NR, SP>;
      else return nullptr;
    case 11:  // the full-capacity class's B -> C -> next A chain, latency form, J in global memory
      if constexpr ((role & 1) != 0) return step_chain<NR, SP, 3>;
      else return nullptr;
    case 12:  // the latency Newton kernel at the throughput register budget (heavy_cap)
      if constexpr ((role & 1) != 0) return step_newton_lat<NR, SP, 1, 1>;
      else return nullptr;
    default:
      return nullptr;
  }
}

}  // namespace mjx
