// tracking_task.hip — fused per-env managers of mjlab's motion-tracking task (gfx950).
//
// The torch managers of Mjlab-Tracking-Flat-Unitree-G1 run ~1,000 small kernels per env
// step; here every manager stage is a handful of launches (include/mjx355_task.h lists the
// reference functions each kernel replaces).  Terminations and rewards run a wave per env
// (lane per command body / joint, wave reductions); command updates, reference-state
// initialisation and push run a thread per env; observations a thread per (env, element).
// Failure-bin sampling statistics are one workgroup.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <stdio.h>

#include <string>

#include "../../include/mjx355_task.h"

namespace mjtr {

constexpr int kPostEnvs = 16;

struct Acc {  // cross-env accumulators of one step's resets (block LDS copy, then global)
  float reward[MJX_TASK_MAX_TERMS];
  float term[MJX_TASK_MAX_TERMS];
  float metric[MJX_TRACK_NMETRIC];
  float count;
};

// ----------------------------------------------------------------------------- math
// quaternions wxyz, as utils/lab_api/math.py (the torch helpers of mjlab_amd/math_utils.py)
struct V3 { float x, y, z; };
struct Q4 { float w, x, y, z; };
__device__ __forceinline__ V3 v3(const float* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ Q4 q4(const float* p) { return {p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float norm3(V3 a) { return sqrtf(dot(a, a)); }
// quat_mul, math.py:526-563 (8-multiply order)
__device__ __forceinline__ Q4 qmul(Q4 a, Q4 b) {
  const float ww = (a.z + a.x) * (b.x + b.y), yy = (a.w - a.y) * (b.w + b.z);
  const float zz = (a.w + a.y) * (b.w - b.z), xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (a.z - a.x) * (b.x - b.y));
  return {qq - ww + (a.z - a.y) * (b.y - b.z), qq - xx + (a.x + a.w) * (b.x + b.w),
          qq - yy + (a.w - a.x) * (b.y + b.z), qq - zz + (a.z + a.y) * (b.w - b.x)};
}
__device__ __forceinline__ Q4 qconj(Q4 q) { return {q.w, -q.x, -q.y, -q.z}; }
// quat_inv: conjugate / max(|q|^2, eps)
__device__ __forceinline__ Q4 qinv(Q4 q) {
  const float s = 1.0f / fmaxf(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z, 1e-9f);
  return {q.w * s, -q.x * s, -q.y * s, -q.z * s};
}
// quat_apply / quat_apply_inverse (math.py:629-670)
__device__ __forceinline__ V3 qapply(Q4 q, V3 v) {
  const V3 u = {q.x, q.y, q.z};
  const V3 t = cross(u, v) * 2.f;
  return v + t * q.w + cross(u, t);
}
__device__ __forceinline__ V3 qapply_inv(Q4 q, V3 v) {
  const V3 u = {q.x, q.y, q.z};
  const V3 t = cross(u, v) * 2.f;
  return v - t * q.w + cross(u, t);
}
// quat_error_magnitude: |axis_angle(q1 * conj(q2))| (math.py:478-506, 688-699)
__device__ __forceinline__ float qerr(Q4 a, Q4 b) {
  Q4 q = qmul(a, qconj(b));
  if (q.w < 0.f) q = {-q.w, -q.x, -q.y, -q.z};
  const float mag = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);
  const float half = atan2f(mag, q.w), ang = 2.f * half;
  const float s = fabsf(ang) > 1e-6f ? sinf(half) / ang : 0.5f - ang * ang / 48.f;
  return mag / fabsf(s);
}
// yaw_quat (math.py:1360)
__device__ __forceinline__ Q4 yaw_only(Q4 q) {
  const float yaw = atan2f(2.f * (q.w * q.z + q.x * q.y), 1.f - 2.f * (q.y * q.y + q.z * q.z));
  return {cosf(0.5f * yaw), 0.f, 0.f, sinf(0.5f * yaw)};
}
// quat_from_euler_xyz (math.py:275-302)
__device__ __forceinline__ Q4 quat_euler(float r, float p, float y) {
  const float cy = cosf(y * 0.5f), sy = sinf(y * 0.5f), cr = cosf(r * 0.5f), sr = sinf(r * 0.5f);
  const float cp = cosf(p * 0.5f), sp = sinf(p * 0.5f);
  return {cy * cr * cp + sy * sr * sp, cy * sr * cp - sy * cr * sp, cy * cr * sp + sy * sr * cp,
          sy * cr * cp - cy * sr * sp};
}
// first two columns of matrix_from_quat, row-major ([:, :2] of the 3x3)
__device__ __forceinline__ void mat2col(Q4 q, float* o) {
  const float w = q.w, x = q.x, y = q.y, z = q.z;
  o[0] = 1 - 2 * (y * y + z * z); o[1] = 2 * (x * y - w * z);
  o[2] = 2 * (x * y + w * z);     o[3] = 1 - 2 * (x * x + z * z);
  o[4] = 2 * (x * z - w * y);     o[5] = 2 * (y * z + w * x);
}

// counter-based uniforms: splitmix64 of (seed, env, step, draw), as velocity_task.hip
__device__ __forceinline__ float urand(uint64_t seed, uint32_t env, uint64_t step, uint32_t draw) {
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(env + 1)) ^
               (0xBF58476D1CE4E5B9ull * (step + 1)) ^ (0x94D049BB133111EBull * (uint64_t)(draw + 1));
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float uniform(float lo, float hi, float u) { return lo + (hi - lo) * u; }
enum : uint32_t { D_RESET_SAMPLE = 0x1000, D_CMD_SAMPLE = 0x2000, D_PUSH = 0x4000,
                  D_NOISE = 0x5000, D_RSI = 0x6000 };

__device__ __forceinline__ float wave_add(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// ----------------------------------------------------------------------------- states
// robot body link state (entity/data.py body_link_*: velocity from cvel about the root's
// subtree com)
struct Link { V3 p, lin, ang; Q4 q; };
__device__ __forceinline__ Link robot_link(const mjxTrackDesc& t, int e, int b) {
  const size_t nb = (size_t)t.nbody;
  Link l;
  l.p = v3(t.xpos + ((size_t)e * nb + b) * 3);
  l.q = q4(t.xquat + ((size_t)e * nb + b) * 4);
  const float* cv = t.cvel + ((size_t)e * nb + b) * 6;
  l.ang = v3(cv);
  const V3 sc = v3(t.subtree_com + ((size_t)e * nb + t.root_body) * 3);
  l.lin = v3(cv + 3) - cross(l.ang, sc - l.p);
  return l;
}
// motion frame of command body k (MotionCommand.body_*_w: positions include the env origin)
__device__ __forceinline__ Link motion_link(const mjxTrackDesc& t, int e, int64_t ts, int k) {
  const size_t i = (size_t)ts * t.nmb + k;
  Link l;
  l.p = v3(t.m_body_pos + 3 * i) + v3(t.env_origins + (size_t)e * 3);
  l.q = q4(t.m_body_quat + 4 * i);
  l.lin = v3(t.m_body_lin + 3 * i);
  l.ang = v3(t.m_body_ang + 3 * i);
  return l;
}
__device__ __forceinline__ int64_t frame_of(const mjxTrackDesc& t, int e) {
  const int64_t ts = t.time_steps[e];
  return ts < 0 ? 0 : (ts >= t.nframe ? t.nframe - 1 : ts);
}

// ----------------------------------------------------------------------------- kernels
// action: thread per (env, joint); target = raw * scale + offset - encoder_bias
__global__ void k_action(const mjxTrackDesc* __restrict__ T, const float* __restrict__ a) {
  const mjxTrackDesc& t = *T;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx == 0) *t.step_counter += 1;
  const int nj = t.njoint;
  if (idx >= t.nworld * nj) return;
  const int e = idx / nj, k = idx - e * nj;
  const size_t i = (size_t)e * nj + k;
  const float raw = a[i];
  t.prev_prev_action[i] = t.prev_action[i];
  t.prev_action[i] = t.action[i];
  t.action[i] = raw;
  float target;
  {
#pragma clang fp contract(off)
    const float scaled = raw * t.action_scale[k];
    const float processed = scaled + t.action_offset[k];
    target = processed - t.encoder_bias[(size_t)e * nj + t.target_of_action[k]];
  }
  t.joint_pos_target[(size_t)e * nj + t.target_of_action[k]] = target;
  t.ctrl[(size_t)e * t.nu + t.ctrl_of_action[k]] = target;
}

// terminations + rewards + reset bookkeeping: wave per env, lane per command body / joint
__device__ __forceinline__ void post_env(const mjxTrackDesc& t, int e, int lane, Acc* acc) {
  const int64_t len = t.episode_length[e] + 1;
  if (lane == 0) t.episode_length[e] = len;
  const int64_t ts = frame_of(t, e);
  const int nmb = t.nmb, nj = t.njoint;
  // per-body squared errors (lane = command body)
  float e_pos = 0.f, e_ori = 0.f, e_lin = 0.f, e_ang = 0.f, e_z = 0.f, e_pn = 0.f;
  if (lane < nmb) {
    const Link r = robot_link(t, e, t.robot_body[lane]);
    const Link m = motion_link(t, e, ts, lane);
    const size_t i = (size_t)e * nmb + lane;
    const V3 rp = v3(t.body_pos_rel + 3 * i);
    const Q4 rq = q4(t.body_quat_rel + 4 * i);
    const V3 dp = rp - r.p;
    e_pos = dot(dp, dp);
    e_pn = sqrtf(e_pos);
    const float qe = qerr(rq, r.q);
    e_ori = qe * qe;
    const V3 dl = m.lin - r.lin, da = m.ang - r.ang;
    e_lin = dot(dl, dl);
    e_ang = dot(da, da);
    e_z = fabsf(rp.z - r.p.z);
  }
  // anchor (motion anchor body vs robot anchor body), every lane
  const Link ra = robot_link(t, e, t.anchor_body);
  const Link ma = motion_link(t, e, ts, t.anchor_motion);
  // joint sums (lane = joint): action rate, soft-limit violation
  float rate = 0.f, lim = 0.f;
  for (int j = lane; j < nj; j += 64) {
    const float da = t.action[(size_t)e * nj + j] - t.prev_action[(size_t)e * nj + j];
    rate += da * da;
    const float q = t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]];
    lim += -fminf(q - t.soft_lo[j], 0.f) + fmaxf(q - t.soft_hi[j], 0.f);
  }
  rate = wave_add(rate);
  lim = wave_add(lim);
  const float* sd = t.sensordata + (size_t)e * t.nsensordata;
  // ---- terminations (termination_manager.py:87-97)
  bool term = false, trunc = false;
  for (int k = 0; k < t.ntermination; k++) {
    const uint32_t bm = t.termination_bodies[k];
    const bool in = lane < nmb && ((bm >> lane) & 1u);
    const float th = t.termination_threshold[k];
    bool v = false;
    switch (t.termination_kind[k]) {
      case MJX_TT_TIME_OUT: v = len >= t.max_episode_length; break;
      case MJX_TT_ANCHOR_POS_Z: v = fabsf(ma.p.z - ra.p.z) > th; break;
      case MJX_TT_ANCHOR_POS: v = norm3(ma.p - ra.p) > th; break;
      case MJX_TT_ANCHOR_ORI: {
        const V3 g = {0.f, 0.f, -1.f};
        v = fabsf(qapply_inv(ma.q, g).z - qapply_inv(ra.q, g).z) > th;
      } break;
      case MJX_TT_BODY_POS_Z: v = __ballot(in && e_z > th) != 0ull; break;
      case MJX_TT_BODY_POS: v = __ballot(in && e_pn > th) != 0ull; break;
    }
    if (lane == 0) t.term_dones[(size_t)k * t.nworld + e] = v;
    if (t.termination_is_timeout[k]) trunc |= v; else term |= v;
  }
  const bool reset = term || trunc;
  if (lane == 0) {
    t.terminated[e] = term;
    t.time_outs[e] = trunc;
    t.reset_buf[e] = reset;
  }
  // ---- rewards (reward_manager.py:77-91), in term order
  const float dt = t.step_dt;
  float total = 0.f;
  for (int k = 0; k < t.nreward; k++) {
    const float w = t.reward_weight[k];
    float* sr = t.step_reward + (size_t)e * t.nreward + k;
    float* es = t.episode_sums + (size_t)k * t.nworld + e;
    if (w == 0.f) {
      if (lane == 0) {
        *sr = 0.f;
        if (reset) { atomicAdd(&acc->reward[k], *es); *es = 0.f; }
      }
      continue;
    }
    const uint32_t bm = t.reward_bodies[k];
    const bool in = lane < nmb && ((bm >> lane) & 1u);
    const float nsel = (float)__popc(bm & (nmb >= 32 ? 0xffffffffu : ((1u << nmb) - 1u)));
    const float s2 = t.reward_std[k] * t.reward_std[k];
    float f = 0.f;
    switch (t.reward_kind[k]) {
      case MJX_TR_ANCHOR_POS: { const V3 d = ma.p - ra.p; f = expf(-dot(d, d) / s2); } break;
      case MJX_TR_ANCHOR_ORI: { const float q = qerr(ma.q, ra.q); f = expf(-q * q / s2); } break;
      case MJX_TR_BODY_POS: f = expf(-(wave_add(in ? e_pos : 0.f) / nsel) / s2); break;
      case MJX_TR_BODY_ORI: f = expf(-(wave_add(in ? e_ori : 0.f) / nsel) / s2); break;
      case MJX_TR_BODY_LIN_VEL: f = expf(-(wave_add(in ? e_lin : 0.f) / nsel) / s2); break;
      case MJX_TR_BODY_ANG_VEL: f = expf(-(wave_add(in ? e_ang : 0.f) / nsel) / s2); break;
      case MJX_TR_ACTION_RATE: f = rate; break;
      case MJX_TR_JOINT_LIMIT: f = lim; break;
      case MJX_TR_SELF_COLLISION: f = sd[t.selfcol_found_adr]; break;
    }
    float v = f * w * dt;
    if (!isfinite(v)) v = 0.f;  // nan_to_num
    total += v;
    if (lane == 0) {
      *sr = v / dt;
      const float es_new = *es + v;
      if (reset) { atomicAdd(&acc->reward[k], es_new); *es = 0.f; }
      else *es = es_new;
    }
  }
  if (lane == 0) t.reward_buf[e] = total;
  if (reset && lane == 0) {
    for (int k = 0; k < t.ntermination; k++)
      if (t.term_dones[(size_t)k * t.nworld + e]) atomicAdd(&acc->term[k], 1.f);
    atomicAdd(&acc->count, 1.f);
  }
  // command metrics of this step's resets (CommandTerm.reset_masked: mean over reset envs)
  if (reset && lane < MJX_TRACK_NMETRIC) atomicAdd(&acc->metric[lane], t.metrics[(size_t)lane * t.nworld + e]);
}

// Accumulators: block LDS copy stored as the block's row of `part` (k_log sums the rows;
// per-field global atomics from every block contend on a few addresses)
constexpr int kAccN = (int)(sizeof(Acc) / sizeof(float));
static_assert(kAccN <= 128, "k_log: thread per accumulator field");
__global__ __launch_bounds__(64 * kPostEnvs) void k_post(const mjxTrackDesc* __restrict__ T,
                                                        float* __restrict__ part) {
  const mjxTrackDesc& t = *T;
  __shared__ Acc sh;
  float* shf = reinterpret_cast<float*>(&sh);
  for (int i = threadIdx.x; i < kAccN; i += blockDim.x) shf[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kPostEnvs + (threadIdx.x >> 6);
  if (e < t.nworld) post_env(t, e, lane, &sh);
  __syncthreads();
  for (int i = threadIdx.x; i < kAccN; i += blockDim.x) part[(size_t)blockIdx.x * kAccN + i] = shf[i];
}

// Failure-bin statistics of one resample (commands.py:258-300), one workgroup: failed
// counts of the masked envs' current bins (overwriting the current counts when any failed),
// sampling probabilities (uniform floor, kernel smoothing with right replicate padding),
// their CDF and the sampling metrics; `ema` then applies _adaptive_update (:301-307).
constexpr int kBinThreads = 256;
__global__ __launch_bounds__(kBinThreads) void k_bins(const mjxTrackDesc* __restrict__ T,
                                                     const uint8_t* __restrict__ mask, int ema) {
  const mjxTrackDesc& t = *T;
  __shared__ float cnt[MJX_TRACK_MAX_BINS];
  __shared__ float pr[MJX_TRACK_MAX_BINS];
  __shared__ int anyfail;
  const int nbin = t.bin_count, tid = threadIdx.x;
  float* cdf = t.sampling;
  if (t.sampling_mode != 2) {  // start / uniform: fixed metrics (commands.py:302-307)
    if (tid == 0) {
      cdf[nbin + 0] = 1.f;
      cdf[nbin + 1] = 1.f / (float)nbin;
      cdf[nbin + 2] = 0.5f;
    }
    return;
  }
  for (int i = tid; i < nbin; i += kBinThreads) cnt[i] = 0.f;
  if (tid == 0) anyfail = 0;
  __syncthreads();
  for (int e = tid; e < t.nworld; e += kBinThreads) {
    if (!mask[e] || !t.terminated[e]) continue;
    int64_t b = (t.time_steps[e] * nbin) / (t.nframe > 1 ? t.nframe : 1);
    b = b < 0 ? 0 : (b >= nbin ? nbin - 1 : b);
    atomicAdd(&cnt[b], 1.f);
    anyfail = 1;
  }
  __syncthreads();
  if (anyfail)
    for (int i = tid; i < nbin; i += kBinThreads) t.current_bin_failed[i] = cnt[i];
  for (int i = tid; i < nbin; i += kBinThreads) {
    float v = 0.f;
    for (int k = 0; k < t.kernel_size; k++) {
      const int j = min(i + k, nbin - 1);
      v += t.kernel[k] * (t.bin_failed_count[j] + t.uniform_ratio / (float)nbin);
    }
    pr[i] = v;
  }
  __syncthreads();
  if (tid == 0) {  // serial over a few bins: normalise, cdf, entropy, argmax
    float s = 0.f;
    for (int i = 0; i < nbin; i++) s += pr[i];
    float c = 0.f, h = 0.f, pmax = -1.f;
    int imax = 0;
    for (int i = 0; i < nbin; i++) {
      const float p = pr[i] / s;
      c += p;
      cdf[i] = c;
      h -= p * logf(p + 1e-12f);
      if (p > pmax) { pmax = p; imax = i; }
    }
    cdf[nbin - 1] = 1.f;
    cdf[nbin + 0] = h / logf((float)nbin);
    cdf[nbin + 1] = pmax;
    cdf[nbin + 2] = (float)imax / (float)nbin;
  }
  __syncthreads();
  if (ema)
    for (int i = tid; i < nbin; i += kBinThreads) {
      t.bin_failed_count[i] = t.bin_failed_count[i] * (1.f - t.adaptive_alpha) +
                              t.adaptive_alpha * t.current_bin_failed[i];
      t.current_bin_failed[i] = 0.f;
    }
}

// MotionCommand._resample_command for the envs of `mask` (commands.py:309-375): start frame
// from the failure-bin CDF (or uniform / 0), then reference-state initialisation: root
// pose / velocity of command body 0 plus the configured noise, joints of the frame plus
// U(joint_position_range) clipped to the soft limits; targets cleared.  `full_reset` adds
// the rest of _reset_idx for the env (action, command-counter, push timer, episode length,
// ctrl).  Every env writes the sampling metrics (CommandTerm fills them for all envs).
// wave per env: lane 0 the sampling, root and counters, lane j joint j
__global__ __launch_bounds__(64 * kPostEnvs) void k_rsi(const mjxTrackDesc* __restrict__ T,
                                                       const uint8_t* __restrict__ mask,
                                                       int full_reset, uint32_t draw) {
  const mjxTrackDesc& t = *T;
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kPostEnvs + (threadIdx.x >> 6);
  if (e >= t.nworld) return;  // wave-uniform
  const int nbin = t.bin_count;
  const float* cdf = t.sampling;
  if (lane < 3) t.metrics[(size_t)(10 + lane) * t.nworld + e] = cdf[nbin + lane];
  if (!mask[e]) return;
  const uint64_t step = *t.step_counter, seed = t.seed;
  const int nj = t.njoint;
  // start frame (every lane draws the same values)
  int64_t ts = 0;
  if (t.sampling_mode == 1) {
    ts = (int64_t)(urand(seed, e, step, draw) * (float)t.nframe);
    ts = ts >= t.nframe ? t.nframe - 1 : ts;
  } else if (t.sampling_mode == 2) {
    const float u = urand(seed, e, step, draw);
    int b = 0;
    while (b < nbin - 1 && cdf[b] <= u) b++;
    ts = (int64_t)(((float)b + urand(seed, e, step, draw + 1)) / (float)nbin * (float)(t.nframe - 1));
  }
  for (int j = lane; j < nj; j += 64) {
    if (full_reset) {
      const size_t i = (size_t)e * nj + j;
      t.action[i] = t.prev_action[i] = t.prev_prev_action[i] = 0.f;
    }
    float jp = t.m_joint_pos[(size_t)ts * nj + j] +
               uniform(t.joint_position_range[0], t.joint_position_range[1], urand(seed, e, step, D_RSI + 12 + j));
    jp = fminf(fmaxf(jp, t.soft_lo[j]), t.soft_hi[j]);
    t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]] = jp;
    t.qvel[(size_t)e * t.nv + t.joint_v_adr[j]] = t.m_joint_vel[(size_t)ts * nj + j];
    t.joint_pos_target[(size_t)e * nj + j] = 0.f;
    if (full_reset)  // Scene.write_data_to_sim after the reset: ctrl <- cleared targets
      t.ctrl[(size_t)e * t.nu + t.ctrl_of_action[j]] = 0.f;
  }
  if (lane != 0) return;
  t.time_steps[e] = ts;
  if (full_reset) {
    t.command_counter[e] = 0;
    if (t.has_push)
      t.push_time_left[e] = uniform(t.push_interval[0], t.push_interval[1], urand(seed, e, step, D_PUSH + 15));
    t.episode_length[e] = 0;
    // CommandTerm._resample_masked: timer and counter (the motion-end resample of
    // _update_command calls _resample_command directly, without them)
    t.command_counter[e] += 1;
    t.time_left[e] = 1e9f;  // resampling_time_range (1e9, 1e9)
  }
  // reference-state initialisation from command body 0
  const Link m = motion_link(t, e, ts, 0);
  float r[6], v[6];
  for (int k = 0; k < 6; k++) {
    r[k] = uniform(t.pose_range[k][0], t.pose_range[k][1], urand(seed, e, step, D_RSI + k));
    v[k] = uniform(t.vel_range[k][0], t.vel_range[k][1], urand(seed, e, step, D_RSI + 6 + k));
  }
  const Q4 qr = qmul(quat_euler(r[3], r[4], r[5]), m.q);
  float* q = t.qpos + (size_t)e * t.nq + t.free_q_adr;
  q[0] = m.p.x + r[0]; q[1] = m.p.y + r[1]; q[2] = m.p.z + r[2];
  q[3] = qr.w; q[4] = qr.x; q[5] = qr.y; q[6] = qr.z;
  const V3 ang_b = qapply_inv(qr, m.ang + V3{v[3], v[4], v[5]});
  float* qv = t.qvel + (size_t)e * t.nv + t.free_v_adr;
  qv[0] = m.lin.x + v[0]; qv[1] = m.lin.y + v[1]; qv[2] = m.lin.z + v[2];
  qv[3] = ang_b.x; qv[4] = ang_b.y; qv[5] = ang_b.z;
}

// CommandTerm.compute, first half: _update_metrics (commands.py:223-257), timer, time step
// advance, envs at the motion end into resample_mask (thread per env)
// Wave per env (kPostEnvs envs per block): lane k takes body k and joint k (a thread-per-env
// loop pays a dependent index-then-state global load per body and joint), wave sums.
__global__ __launch_bounds__(64 * kPostEnvs) void k_cmd(const mjxTrackDesc* __restrict__ T) {
  const mjxTrackDesc& t = *T;
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kPostEnvs + (threadIdx.x >> 6);
  if (e >= t.nworld) return;  // wave-uniform
  const int64_t ts = frame_of(t, e);
  const int nmb = t.nmb, nj = t.njoint;
  float* M = t.metrics;
  const size_t N = (size_t)t.nworld;
  float bp = 0.f, bo = 0.f, bl = 0.f, ba = 0.f;
  for (int k = lane; k < nmb; k += 64) {
    const Link r = robot_link(t, e, t.robot_body[k]), m = motion_link(t, e, ts, k);
    const size_t i = (size_t)e * nmb + k;
    bp += norm3(v3(t.body_pos_rel + 3 * i) - r.p);
    bo += qerr(q4(t.body_quat_rel + 4 * i), r.q);
    bl += norm3(m.lin - r.lin);
    ba += norm3(m.ang - r.ang);
  }
  float jp = 0.f, jv = 0.f;
  for (int j = lane; j < nj; j += 64) {
    const float dp = t.m_joint_pos[(size_t)ts * nj + j] - t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]];
    const float dv = t.m_joint_vel[(size_t)ts * nj + j] - t.qvel[(size_t)e * t.nv + t.joint_v_adr[j]];
    jp += dp * dp;
    jv += dv * dv;
  }
  bp = wave_add(bp); bo = wave_add(bo); bl = wave_add(bl); ba = wave_add(ba);
  jp = wave_add(jp); jv = wave_add(jv);
  if (lane != 0) return;
  const Link ra = robot_link(t, e, t.anchor_body), ma = motion_link(t, e, ts, t.anchor_motion);
  M[0 * N + e] = norm3(ma.p - ra.p);
  M[1 * N + e] = qerr(ma.q, ra.q);
  M[2 * N + e] = norm3(ma.lin - ra.lin);
  M[3 * N + e] = norm3(ma.ang - ra.ang);
  M[4 * N + e] = bp / (float)nmb;
  M[5 * N + e] = bo / (float)nmb;
  M[6 * N + e] = bl / (float)nmb;
  M[7 * N + e] = ba / (float)nmb;
  M[8 * N + e] = sqrtf(jp);
  M[9 * N + e] = sqrtf(jv);
  t.time_left[e] -= t.step_dt;
  const int64_t nts = t.time_steps[e] + 1;
  t.time_steps[e] = nts;
  t.resample_mask[e] = nts >= t.nframe;
}

// _relative_targets (commands.py:384-404) after the resample, then the interval push
// (event_manager.py:124-146, events.py:209-223); thread per env
__global__ __launch_bounds__(64 * kPostEnvs) void k_targets(const mjxTrackDesc* __restrict__ T) {
  // wave per env, lane per body (the stores of a thread-per-env loop may alias the next
  // body's loads, which then serialise)
  const mjxTrackDesc& t = *T;
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kPostEnvs + (threadIdx.x >> 6);
  if (e >= t.nworld) return;  // wave-uniform
  const int64_t ts = frame_of(t, e);
  const int nmb = t.nmb;
  const Link ra = robot_link(t, e, t.anchor_body), ma = motion_link(t, e, ts, t.anchor_motion);
  const V3 dpos = {ra.p.x, ra.p.y, ma.p.z};
  const Q4 dori = yaw_only(qmul(ra.q, qinv(ma.q)));
  for (int k = lane; k < nmb; k += 64) {
    const Link m = motion_link(t, e, ts, k);
    const size_t i = (size_t)e * nmb + k;
    const Q4 q = qmul(dori, m.q);
    const V3 p = dpos + qapply(dori, m.p - ma.p);
    float* op = t.body_pos_rel + 3 * i;
    float* oq = t.body_quat_rel + 4 * i;
    op[0] = p.x; op[1] = p.y; op[2] = p.z;
    oq[0] = q.w; oq[1] = q.x; oq[2] = q.y; oq[3] = q.z;
  }
  if (lane == 0 && t.has_push) {
    float pt = t.push_time_left[e] - t.step_dt;
    if (pt < 1e-6f) {
      const uint64_t step = *t.step_counter, seed = t.seed;
      pt = uniform(t.push_interval[0], t.push_interval[1], urand(seed, e, step, D_PUSH));
      float u[6];
      for (int i = 0; i < 6; i++)
        u[i] = uniform(t.push_vel_range[i][0], t.push_vel_range[i][1], urand(seed, e, step, D_PUSH + 1 + i));
      const Link r = robot_link(t, e, t.root_body);
      float* v = t.qvel + (size_t)e * t.nv + t.free_v_adr;
      const Q4 qq = q4(t.qpos + (size_t)e * t.nq + t.free_q_adr + 3);
      const V3 ang_b = qapply_inv(qq, r.ang + V3{u[3], u[4], u[5]});
      v[0] = r.lin.x + u[0]; v[1] = r.lin.y + u[1]; v[2] = r.lin.z + u[2];
      v[3] = ang_b.x; v[4] = ang_b.y; v[5] = ang_b.z;
    }
    t.push_time_left[e] = pt;
  }
}

// observations: thread per (env, critic element); the policy elements are the critic's
// shared terms (+ noise) with the biased joint positions
__global__ void k_obs(const mjxTrackDesc* __restrict__ T) {
  const mjxTrackDesc& t = *T;
  const int nj = t.njoint, nmb = t.nmb;
  const int nel = t.ncritic;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= t.nworld * nel) return;
  const int e = idx / nel;
  int i = idx - e * nel;
  const int64_t ts = frame_of(t, e);
  const float* sd = t.sensordata + (size_t)e * t.nsensordata;
  // critic layout: [cmd 2nj | apos 3 | aori 6 | body_pos 3nmb | body_ori 6nmb | lin 3 | ang 3 | jpos nj | jvel nj | act nj]
  const int o_apos = 2 * nj, o_aori = o_apos + 3, o_bpos = o_aori + 6, o_bori = o_bpos + 3 * nmb;
  const int o_lin = o_bori + 6 * nmb, o_ang = o_lin + 3, o_jp = o_ang + 3, o_jv = o_jp + nj, o_act = o_jv + nj;
  float val, noise = 0.f;
  int pol = -1;  // policy element index
  // policy layout: [cmd 2nj | apos 3? | aori 6 | lin 3? | ang 3 | jpos nj | jvel nj | act nj]
  const int p_apos = 2 * nj, p_aori = p_apos + (t.policy_anchor_pos ? 3 : 0), p_lin = p_aori + 6;
  const int p_ang = p_lin + (t.policy_lin_vel ? 3 : 0), p_jp = p_ang + 3, p_jv = p_jp + nj, p_act = p_jv + nj;
  float pol_val = 0.f;
  if (i < o_apos) {
    val = i < nj ? t.m_joint_pos[(size_t)ts * nj + i] : t.m_joint_vel[(size_t)ts * nj + i - nj];
    pol = i;
    pol_val = val;
  } else if (i < o_bpos) {
    const Link ra = robot_link(t, e, t.anchor_body), ma = motion_link(t, e, ts, t.anchor_motion);
    const Q4 qi = qinv(ra.q);
    if (i < o_aori) {
      const V3 p = qapply(qi, ma.p - ra.p);
      const int c = i - o_apos;
      val = c == 0 ? p.x : (c == 1 ? p.y : p.z);
      if (t.policy_anchor_pos) { pol = p_apos + c; noise = t.noise_anchor_pos; }
    } else {
      float m6[6];
      mat2col(qmul(qi, ma.q), m6);
      const int c = i - o_aori;
      val = m6[c];
      pol = p_aori + c;
      noise = t.noise_anchor_ori;
    }
    pol_val = val;
  } else if (i < o_lin) {
    const Link ra = robot_link(t, e, t.anchor_body);
    const Q4 qi = qinv(ra.q);
    if (i < o_bori) {
      const int k = (i - o_bpos) / 3, c = (i - o_bpos) % 3;
      const V3 p = qapply(qi, robot_link(t, e, t.robot_body[k]).p - ra.p);
      val = c == 0 ? p.x : (c == 1 ? p.y : p.z);
    } else {
      const int k = (i - o_bori) / 6, c = (i - o_bori) % 6;
      float m6[6];
      mat2col(qmul(qi, robot_link(t, e, t.robot_body[k]).q), m6);
      val = m6[c];
    }
  } else if (i < o_ang) {
    val = sd[t.imu_lin_vel_adr + i - o_lin];
    if (t.policy_lin_vel) { pol = p_lin + i - o_lin; noise = t.noise_lin_vel; pol_val = val; }
  } else if (i < o_jp) {
    val = sd[t.imu_ang_vel_adr + i - o_ang];
    pol = p_ang + i - o_ang; noise = t.noise_ang_vel; pol_val = val;
  } else if (i < o_jv) {
    const int j = i - o_jp;
    const float q = t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]];
    val = q - t.default_joint_pos[j];
    pol = p_jp + j; noise = t.noise_joint_pos;
    pol_val = (q + t.encoder_bias[(size_t)e * nj + j]) - t.default_joint_pos[j];  // biased
  } else if (i < o_act) {
    const int j = i - o_jv;
    val = t.qvel[(size_t)e * t.nv + t.joint_v_adr[j]];
    pol = p_jv + j; noise = t.noise_joint_vel; pol_val = val;
  } else {
    val = t.action[(size_t)e * nj + i - o_act];
    pol = p_act + i - o_act; pol_val = val;
  }
  t.obs_critic[(size_t)e * nel + i] = val;
  if (pol >= 0) {
    if (t.corrupt_policy && noise > 0.f)
      pol_val += uniform(-noise, noise, urand(t.seed, e, *t.step_counter, D_NOISE + pol));
    t.obs_policy[(size_t)e * t.npolicy + pol] = pol_val;
  }
}

// episode logs of the step's resets (k_post's accumulators), then cleared
constexpr int kLogChunks = 8;
__global__ __launch_bounds__(128 * kLogChunks) void k_log(const mjxTrackDesc* __restrict__ T,
                                                          const float* __restrict__ part, int nblock) {
  const mjxTrackDesc& t = *T;
  __shared__ Acc sh;
  __shared__ float red[kLogChunks][128];
  // column sums of k_post's block rows: 8 row chunks x 128 field lanes, then an LDS fold
  const int i = threadIdx.x & 127, c = threadIdx.x >> 7;
  float sum = 0.f;
  if (i < kAccN) {
    const int per = (nblock + kLogChunks - 1) / kLogChunks;
    const int b0 = c * per, b1 = min(nblock, b0 + per);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int b = b0;
    for (; b + 7 < b1; b += 8)
#pragma unroll
      for (int u = 0; u < 8; u++) s[u] += part[(size_t)(b + u) * kAccN + i];
    for (; b < b1; b++) s[0] += part[(size_t)b * kAccN + i];
    sum = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  }
  red[c][i] = sum;
  __syncthreads();
  if (c == 0 && i < kAccN) {
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < kLogChunks; k++) tot += red[k][i];
    reinterpret_cast<float*>(&sh)[i] = tot;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const Acc& acc = sh;
  if (acc.count > 0.f) {
    for (int k = 0; k < t.nreward; k++) t.log_reward[k] = acc.reward[k] / acc.count / t.episode_length_s;
    for (int k = 0; k < t.ntermination; k++) t.log_termination[k] = acc.term[k];
    for (int k = 0; k < MJX_TRACK_NMETRIC; k++) t.log_metric[k] = acc.metric[k] / acc.count;
  }
}

}  // namespace mjtr

// ----------------------------------------------------------------------------- C ABI
struct mjxTrack_ {
  mjxTrackDesc host;
  mjxTrackDesc* dev = nullptr;
  float* part = nullptr;  // [nblock][kAccN] k_post block partials
  int nworld = 0;
};

static thread_local std::string g_track_err;
static int track_fail(const std::string& s) {
  g_track_err = s;
  return -1;
}
static int track_launched(const char* what) {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : track_fail(std::string(what) + ": " + hipGetErrorString(e));
}

// The tracking descriptor's indices and kinds against its declared sizes (as validate_task in
// velocity_task.hip): a mismatch is an error code, never a device fault.
static std::string validate_track(const mjxTrackDesc& t) {
  auto in = [](int v, int n) { return v >= 0 && v < n; };
  auto span = [](int adr, int len, int n) { return adr >= 0 && adr + len <= n; };
  char buf[256];
  auto err = [&](const char* fmt, int a, int b) {
    snprintf(buf, sizeof buf, fmt, a, b);
    return std::string(buf);
  };
  if (t.nworld <= 0 || t.nq <= 0 || t.nv <= 0 || t.nu <= 0 || t.nbody <= 0 || t.nsensordata < 0)
    return "non-positive model or batch size";
  if (t.njoint < 1) return "no joints";
  const void* need[] = {t.qpos, t.qvel, t.ctrl, t.xpos, t.xquat, t.cvel, t.subtree_com, t.sensordata,
                        t.encoder_bias, t.env_origins, t.m_joint_pos, t.m_joint_vel, t.m_body_pos,
                        t.m_body_quat, t.m_body_lin, t.m_body_ang, t.action, t.prev_action,
                        t.prev_prev_action, t.joint_pos_target, t.episode_length, t.time_steps,
                        t.body_pos_rel, t.body_quat_rel, t.bin_failed_count, t.current_bin_failed,
                        t.sampling, t.metrics, t.time_left, t.command_counter, t.episode_sums,
                        t.step_reward, t.reward_buf, t.reset_buf, t.terminated, t.time_outs,
                        t.term_dones, t.resample_mask, t.obs_policy, t.obs_critic, t.log_reward,
                        t.log_termination, t.log_metric, t.step_counter};
  for (size_t i = 0; i < sizeof need / sizeof need[0]; i++)
    if (!need[i]) return err("required buffer %d of the descriptor is null", (int)i, 0);
  if (t.has_push && !t.push_time_left) return "has_push without push_time_left";
  if (!in(t.root_body, t.nbody)) return err("root_body %d outside [0, %d)", t.root_body, t.nbody);
  if (!span(t.free_q_adr, 7, t.nq)) return err("free joint qpos %d + 7 past nq %d", t.free_q_adr, t.nq);
  if (!span(t.free_v_adr, 6, t.nv)) return err("free joint qvel %d + 6 past nv %d", t.free_v_adr, t.nv);
  for (int j = 0; j < t.njoint; j++) {
    if (!in(t.joint_q_adr[j], t.nq)) return err("joint %d qpos address outside [0, nq=%d)", j, t.nq);
    if (!in(t.joint_v_adr[j], t.nv)) return err("joint %d qvel address outside [0, nv=%d)", j, t.nv);
    if (!in(t.ctrl_of_action[j], t.nu)) return err("action %d ctrl index outside [0, nu=%d)", j, t.nu);
    if (!in(t.target_of_action[j], t.njoint))
      return err("action %d target column outside [0, njoint=%d)", j, t.njoint);
  }
  for (int k = 0; k < t.nmb; k++)
    if (!in(t.robot_body[k], t.nbody)) return err("command body %d: model body outside [0, %d)", k, t.nbody);
  if (!in(t.anchor_motion, t.nmb)) return err("anchor_motion %d outside [0, nmb=%d)", t.anchor_motion, t.nmb);
  if (!in(t.anchor_body, t.nbody)) return err("anchor_body %d outside [0, %d)", t.anchor_body, t.nbody);
  if (!span(t.imu_lin_vel_adr, 3, t.nsensordata) || !span(t.imu_ang_vel_adr, 3, t.nsensordata))
    return err("imu velocity sensors (%d, %d) + 3 past nsensordata", t.imu_lin_vel_adr, t.imu_ang_vel_adr);
  if (t.selfcol_found_adr >= t.nsensordata)
    return err("self-collision sensor %d outside [-1, %d)", t.selfcol_found_adr, t.nsensordata);
  if (t.max_episode_length <= 0 || !(t.step_dt > 0.f)) return "non-positive episode length or step_dt";
  if (t.sampling_mode < 0 || t.sampling_mode > 2) return err("unknown sampling_mode %d", t.sampling_mode, 0);
  const uint32_t body_bits = t.nmb >= 32 ? 0xffffffffu : (1u << t.nmb) - 1u;
  for (int k = 0; k < t.nreward; k++) {
    const int kind = t.reward_kind[k];
    if (!in(kind, MJX_TR_SELF_COLLISION + 1)) return err("reward %d: unknown kind %d", k, kind);
    if (kind == MJX_TR_SELF_COLLISION && t.selfcol_found_adr < 0)
      return err("reward %d: kind %d needs selfcol_found_adr", k, kind);
    if (t.reward_bodies[k] & ~body_bits) return err("reward %d: body mask past nmb %d", k, t.nmb);
  }
  for (int k = 0; k < t.ntermination; k++) {
    const int kind = t.termination_kind[k];
    if (!in(kind, MJX_TT_BODY_POS + 1)) return err("termination %d: unknown kind %d", k, kind);
    if (t.termination_bodies[k] & ~body_bits) return err("termination %d: body mask past nmb %d", k, t.nmb);
  }
  return "";
}

extern "C" {

size_t mjx_track_desc_size(void) { return sizeof(mjxTrackDesc); }

int mjx_track_create(const mjxTrackDesc* d, mjxTrack** out) {
  if (!d || !out) return track_fail("null argument");
  if (d->njoint > MJX_TASK_MAX_JOINTS || d->nmb > MJX_TRACK_MAX_BODIES || d->nmb < 1 ||
      d->nreward > MJX_TASK_MAX_TERMS || d->ntermination > MJX_TASK_MAX_TERMS ||
      d->bin_count < 1 || d->bin_count > MJX_TRACK_MAX_BINS || d->kernel_size < 1 ||
      d->kernel_size > 8 || d->nframe < 1)
    return track_fail("tracking descriptor exceeds compiled capacities");
  const int nj = d->njoint, nmb = d->nmb;
  if (d->ncritic != 5 * nj + 9 * nmb + 15 ||
      d->npolicy != 5 * nj + 9 + (d->policy_anchor_pos ? 3 : 0) + (d->policy_lin_vel ? 3 : 0))
    return track_fail("observation sizes do not match the tracking layout");
  {
    const std::string why = validate_track(*d);
    if (!why.empty()) return track_fail("mjx_track_create: " + why);
  }
  auto* t = new mjxTrack_();
  t->host = *d;
  t->nworld = d->nworld;
  if (hipMalloc((void**)&t->dev, sizeof(mjxTrackDesc)) != hipSuccess ||
      hipMalloc((void**)&t->part, sizeof(float) * mjtr::kAccN *
                ((t->nworld + mjtr::kPostEnvs - 1) / mjtr::kPostEnvs + 1)) != hipSuccess) {
    delete t;
    return track_fail("hipMalloc failed");
  }
  if (hipMemcpy(t->dev, d, sizeof(mjxTrackDesc), hipMemcpyHostToDevice) != hipSuccess) {
    delete t;
    return track_fail("upload failed");
  }
  *out = t;
  return 0;
}

int mjx_track_destroy(mjxTrack* t) {
  if (!t) return 0;
  if (t->dev) (void)hipFree(t->dev);
  if (t->part) (void)hipFree(t->part);
  delete t;
  return 0;
}

int mjx_track_action(mjxTrack* t, const float* action, void* stream) {
  if (!t) return track_fail("null task");
  const long n = (long)t->nworld * t->host.njoint;
  hipLaunchKernelGGL(mjtr::k_action, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, t->dev, action);
  return track_launched("k_action");
}

int mjx_track_post(mjxTrack* t, void* stream) {
  if (!t) return track_fail("null task");
  hipLaunchKernelGGL(mjtr::k_post, dim3((t->nworld + mjtr::kPostEnvs - 1) / mjtr::kPostEnvs),
                     dim3(64 * mjtr::kPostEnvs), 0, (hipStream_t)stream, t->dev, t->part);
  hipLaunchKernelGGL(mjtr::k_log, dim3(1), dim3(128 * mjtr::kLogChunks), 0, (hipStream_t)stream, t->dev, t->part,
                     (t->nworld + mjtr::kPostEnvs - 1) / mjtr::kPostEnvs);
  return track_launched("k_post");
}

int mjx_track_reset(mjxTrack* t, void* stream) {
  if (!t) return track_fail("null task");
  const int nwave = (t->nworld + mjtr::kPostEnvs - 1) / mjtr::kPostEnvs;  // blocks of kPostEnvs waves
  hipLaunchKernelGGL(mjtr::k_bins, dim3(1), dim3(mjtr::kBinThreads), 0, (hipStream_t)stream,
                     t->dev, (const uint8_t*)t->host.reset_buf, 0);
  hipLaunchKernelGGL(mjtr::k_rsi, dim3(nwave), dim3(64 * mjtr::kPostEnvs), 0, (hipStream_t)stream,
                     t->dev, (const uint8_t*)t->host.reset_buf, 1, (uint32_t)mjtr::D_RESET_SAMPLE);
  return track_launched("k_rsi");
}

int mjx_track_observe(mjxTrack* t, void* stream) {
  if (!t) return track_fail("null task");
  const int nwave = (t->nworld + mjtr::kPostEnvs - 1) / mjtr::kPostEnvs;  // blocks of kPostEnvs waves
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mjtr::k_cmd, dim3(nwave), dim3(64 * mjtr::kPostEnvs), 0, s, t->dev);
  hipLaunchKernelGGL(mjtr::k_bins, dim3(1), dim3(mjtr::kBinThreads), 0, s, t->dev,
                     (const uint8_t*)t->host.resample_mask, 1);
  hipLaunchKernelGGL(mjtr::k_rsi, dim3(nwave), dim3(64 * mjtr::kPostEnvs), 0, s, t->dev,
                     (const uint8_t*)t->host.resample_mask, 0, (uint32_t)mjtr::D_CMD_SAMPLE);
  hipLaunchKernelGGL(mjtr::k_targets, dim3(nwave), dim3(64 * mjtr::kPostEnvs), 0, s, t->dev);
  const long n = (long)t->nworld * t->host.ncritic;
  hipLaunchKernelGGL(mjtr::k_obs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, t->dev);
  return track_launched("k_obs");
}

const char* mjx_track_last_error(void) { return g_track_err.c_str(); }

}  // extern "C"
