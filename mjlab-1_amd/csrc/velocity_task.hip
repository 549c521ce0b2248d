// velocity_task.hip — fused per-env managers of mjlab's velocity tasks (gfx950).
//
// One thread per env; every manager stage of ManagerBasedRlEnv.step() that the torch
// stack runs as ~700 small kernels per env step becomes one of five launches (see
// include/mjx355_task.h for the reference functions each kernel replaces).  The work is
// a few hundred flops per env against ~1-2 KB of per-env state, so the kernels are
// latency-bound; they read the mjx355 data arena and write the managers' torch tensors
// in place.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "../../include/mjx355_task.h"

namespace mjxt {

constexpr int kBlock = 128;

struct Acc {  // device accumulators, reduced across envs with atomics
  float reward[MJX_TASK_MAX_TERMS];
  float term[MJX_TASK_MAX_TERMS];
  float cmd[2];
  float metric_sum[MJX_MT_COUNT];
  float metric_cnt[MJX_MT_COUNT];
  float count;
};

struct V3 { float x, y, z; };
__device__ __forceinline__ V3 v3(const float* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// quaternions (w, x, y, z): utils/lab_api/math.py quat_apply(_inverse) :629-670
__device__ __forceinline__ V3 qrot(const float* q, V3 v, float sgn) {
  const float w = q[0];
  V3 u = {sgn * q[1], sgn * q[2], sgn * q[3]};
  V3 t = cross(u, v);
  t = {2.f * t.x, 2.f * t.y, 2.f * t.z};
  V3 c = cross(u, t);
  return {v.x + w * t.x + c.x, v.y + w * t.y + c.y, v.z + w * t.z + c.z};
}
__device__ __forceinline__ V3 qapply(const float* q, V3 v) { return qrot(q, v, 1.f); }
__device__ __forceinline__ V3 qapply_inv(const float* q, V3 v) { return qrot(q, v, -1.f); }
__device__ __forceinline__ void qmul(const float* a, const float* b, float* r) {
  r[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  r[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  r[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  r[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}
// quat_from_euler_xyz (math.py:275-302)
__device__ __forceinline__ void quat_euler(float r, float p, float y, float* q) {
  float cy = cosf(y * 0.5f), sy = sinf(y * 0.5f), cr = cosf(r * 0.5f), sr = sinf(r * 0.5f);
  float cp = cosf(p * 0.5f), sp = sinf(p * 0.5f);
  q[0] = cy * cr * cp + sy * sr * sp;
  q[1] = cy * sr * cp - sy * cr * sp;
  q[2] = cy * cr * sp + sy * sr * cp;
  q[3] = sy * cr * cp - cy * sr * sp;
}
__device__ __forceinline__ float wrap_to_pi(float a) {
  const float tp = 6.283185307179586f;
  float w = fmodf(a + 3.141592653589793f, tp);
  if (w < 0.f) w += tp;
  return w - 3.141592653589793f;
}

// counter-based uniform randoms: splitmix64 of (seed, env, step, draw)
__device__ __forceinline__ float urand(uint64_t seed, uint32_t env, uint64_t step, uint32_t draw) {
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(env + 1)) ^
               (0xBF58476D1CE4E5B9ull * (step + 1)) ^ (0x94D049BB133111EBull * (uint64_t)(draw + 1));
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);  // [0, 1)
}
__device__ __forceinline__ float uniform(float lo, float hi, float u) { return lo + (hi - lo) * u; }

// draw ids (per env, per env-step), kept disjoint between kernels
enum : uint32_t { D_RESET = 0x1000, D_CMD_RESET = 0x2000, D_CMD = 0x3000, D_PUSH = 0x4000,
                  D_NOISE = 0x5000, D_TERRAIN = 0x6000 };

// EntityData derived reads (entity/data.py:20-31, 219-229, 320-327)
struct Root {
  V3 lin_w, ang_w, lin_b, ang_b, grav_b;
  const float* quat;
};
__device__ __forceinline__ Root root_state(const mjxTaskDesc& t, int e) {
  Root r;
  const int b = t.root_body;
  const size_t nb = (size_t)t.nbody;
  const float* cv = t.cvel + ((size_t)e * nb + b) * 6;
  V3 ang = v3(cv), linc = v3(cv + 3);
  V3 off = sub(v3(t.subtree_com + ((size_t)e * nb + b) * 3), v3(t.xpos + ((size_t)e * nb + b) * 3));
  V3 c = cross(ang, off);
  r.lin_w = sub(linc, c);
  r.ang_w = ang;
  r.quat = t.xquat + ((size_t)e * nb + b) * 4;
  r.lin_b = qapply_inv(r.quat, r.lin_w);
  r.ang_b = qapply_inv(r.quat, r.ang_w);
  r.grav_b = qapply_inv(r.quat, V3{0.f, 0.f, -1.f});
  return r;
}
// site velocity (world, linear part) with the entity root's subtree com
__device__ __forceinline__ V3 site_lin_vel(const mjxTaskDesc& t, int e, int site, int body) {
  const size_t nb = (size_t)t.nbody;
  const float* cv = t.cvel + ((size_t)e * nb + body) * 6;
  V3 sc = v3(t.subtree_com + ((size_t)e * nb + t.root_body) * 3);
  V3 p = v3(t.site_xpos + ((size_t)e * t.nsite + site) * 3);
  return sub(v3(cv + 3), cross(v3(cv), sub(sc, p)));
}
__device__ __forceinline__ float command_active(const float* c, float thr) {
  return (sqrtf(c[0] * c[0] + c[1] * c[1]) + fabsf(c[2])) > thr ? 1.f : 0.f;
}
// reward-term command gate: the twist command's activity, or none (command_name None, p_nocmd)
__device__ __forceinline__ float command_gate(const mjxTaskDesc& t, const float* c, float thr,
                                              float p_nocmd) {
  return (t.command_kind != MJX_CMD_TWIST || p_nocmd > 0.5f) ? 1.f : command_active(c, thr);
}

// ----------------------------------------------------------------------------- kernels
// Thread per (env, joint): a thread-per-env loop serialises every iteration on a global
// load, since its stores may alias the next iteration's loads.
__global__ void k_action(const mjxTaskDesc* __restrict__ T, const float* __restrict__ a) {
  const mjxTaskDesc& t = *T;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx == 0) *t.step_counter += 1;  // later kernels of this env step read the new value
  const int nj = t.njoint;
  if (idx >= t.nworld * nj) return;
  const int e = idx / nj, k = idx - e * nj;
  {
    const size_t i = (size_t)e * nj + k;
    const float raw = a[i];
    t.prev_prev_action[i] = t.prev_action[i];
    t.prev_action[i] = t.action[i];
    t.action[i] = raw;
    // separately rounded mul + add, as torch computes raw * scale + offset (no FMA), so
    // ctrl is bitwise identical to the torch manager path
    float target;
    {
#pragma clang fp contract(off)
      const float scaled = raw * t.action_scale[k];
      target = scaled + t.action_offset[k];
    }
    t.joint_pos_target[(size_t)e * nj + t.target_of_action[k]] = target;
    t.ctrl[(size_t)e * t.nu + t.ctrl_of_action[k]] = target;
  }
}

__global__ void k_substep(const mjxTaskDesc* __restrict__ T) {
  const mjxTaskDesc& t = *T;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= t.nworld) return;
  const float now = t.time[e];
  const float el = now - t.last_time[e];
  for (int f = 0; f < t.nfeet; f++) {
    const size_t i = (size_t)e * t.nfeet + f;
    const bool contact = t.sensordata[(size_t)e * t.nsensordata + t.feet_found_adr[f]] > 0.f;
    const float ca = t.cur_air[i], cc = t.cur_contact[i];
    if (ca > 0.f && contact) t.last_air[i] = ca + el;
    t.cur_air[i] = contact ? 0.f : ca + el;
    if (cc > 0.f && !contact) t.last_contact[i] = cc + el;
    t.cur_contact[i] = contact ? cc + el : 0.f;
  }
  t.last_time[e] = now;
}

// Per-env terminations, rewards and reset bookkeeping.  Cross-env accumulators go to the
// block's LDS copy of Acc (ds_add_f32) and are flushed with one global atomic per field and
// block: thousands of lanes adding into the same few global addresses serialise at the
// memory side (MI355X_MICROARCH.md, float atomics: one target row is ~14x slower).
// Joint sums of the per-joint reward terms, reduced over the env's wave (lane per joint):
// pose deviation under each std table, soft-limit violation, action rate.  A thread-per-env
// loop pays two dependent global loads (joint index, then qpos) per joint.
struct JointSums { float pose[3], lim, rate, acc2, torque2, power, jv_var; };
__device__ __forceinline__ float wave_add(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ JointSums joint_sums(const mjxTaskDesc& t, int e, int lane) {
  JointSums r{{0.f, 0.f, 0.f}, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int nj = t.njoint;
  if (t.command_kind == MJX_CMD_JUMP) {
    // jump terms (tasks/jump/mdp/rewards.py): action acceleration, actuator torques,
    // explosive_takeoff's |actuator_force[i] * joint_vel[i]| (actuator i paired with joint i,
    // as the reference's element-wise product), joint-velocity variance (two passes)
    // nj <= 64 (mjx_task_create): lane j holds joint j, straight-line code so the loads of
    // the env's joints issue together
    float jv = 0.f;
    if (lane < nj) {
      const int j = lane;
      const size_t i = (size_t)e * nj + j;
      const float a2 = t.action[i] - 2.f * t.prev_action[i] + t.prev_prev_action[i];
      r.acc2 = a2 * a2;
      const float f = t.actuator_force[(size_t)e * t.nu + t.act_ctrl[j]];
      r.torque2 = f * f;
      jv = t.qvel[(size_t)e * t.nv + t.joint_v_adr[j]];
      if ((t.explosive_joints >> j) & 1ull) r.power = fabsf(f * jv);
    }
    const float jv_mean = wave_add(jv) / (float)nj;
    if (lane < nj) {
      const float d = jv - jv_mean;
      r.jv_var = d * d;
    }
    r.acc2 = wave_add(r.acc2);
    r.torque2 = wave_add(r.torque2);
    r.power = wave_add(r.power);
    r.jv_var = wave_add(r.jv_var) / (float)nj;
  }
  if (lane < nj) {
    const int j = lane;
    const float q = t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]];
    const float d = q - t.default_joint_pos[j];
    const float s0 = t.std_standing[j], s1 = t.std_walking[j], s2 = t.std_running[j];
    r.pose[0] = d * d / (s0 * s0);
    r.pose[1] = d * d / (s1 * s1);
    r.pose[2] = d * d / (s2 * s2);
    r.lim = fmaxf(t.soft_lo[j] - q, 0.f) + fmaxf(q - t.soft_hi[j], 0.f);
    const float da = t.action[(size_t)e * nj + j] - t.prev_action[(size_t)e * nj + j];
    r.rate = da * da;
  }
  for (int k = 0; k < 3; k++) r.pose[k] = wave_add(r.pose[k]);
  r.lim = wave_add(r.lim);
  r.rate = wave_add(r.rate);
  return r;
}

// Per-foot values of one env, staged lane-parallel (lane s = foot s) before the term switch:
// the terms' lanes diverge, so every global load inside a case runs in that case's own
// serial turn -- loaded up front they overlap, and the cases read LDS.
struct FootVals { float found, z, vx, vy, air, cc, peak, fx, fy, fz; };
struct EnvVals {
  FootVals f[MJX_TASK_MAX_FEET];
  float og_x, og_y, ocv0, ocv1;  // orient body: projected gravity xy, angular velocity xy
  int illegal;                   // any illegal-contact slot found
};
__device__ __forceinline__ void stage_env(const mjxTaskDesc& t, const int e, const Root& r,
                                          const float* sd, const int lane, EnvVals* ev) {
  if (lane < t.nfeet) {
    const int s = lane;
    const size_t i = (size_t)e * t.nfeet + s;
    FootVals f;
    f.found = sd[t.feet_found_adr[s]];
    const float* fv = sd + t.feet_force_adr[s];
    f.fx = fv[0]; f.fy = fv[1]; f.fz = fv[2];
    f.z = t.site_xpos[((size_t)e * t.nsite + t.foot_site[s]) * 3 + 2];
    const V3 v = site_lin_vel(t, e, t.foot_site[s], t.foot_site_body[s]);
    f.vx = v.x; f.vy = v.y;
    f.air = t.cur_air[i]; f.cc = t.cur_contact[i]; f.peak = t.peak_heights[i];
    ev->f[s] = f;
  }
  const bool ill = lane < t.nillegal && sd[t.illegal_found_adr[lane]] > 0.f;
  const unsigned long long ib = __ballot(ill);
  if (lane == 0) {
    ev->illegal = ib != 0ull;
    V3 g = r.grav_b;
    float c0 = 0.f, c1 = 0.f;
    if (t.orient_body >= 0) {
      g = qapply_inv(t.xquat + ((size_t)e * t.nbody + t.orient_body) * 4, V3{0.f, 0.f, -1.f});
      const float* cv = t.cvel + ((size_t)e * t.nbody + t.orient_body) * 6;
      c0 = cv[0]; c1 = cv[1];
    }
    ev->og_x = g.x; ev->og_y = g.y; ev->ocv0 = c0; ev->ocv1 = c1;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Called by every lane of the env's wave: lane k evaluates termination k and reward term k
// (terms are independent; their loads overlap instead of queueing behind each other's
// stores), the wave reduces the flags and the reward total.
__device__ __forceinline__ void post_env(const mjxTaskDesc& t, const int e, const JointSums& js,
                                         const int lane, Acc* __restrict__ acc,
                                         EnvVals* __restrict__ ev) {
  const int64_t len = t.episode_length[e] + 1;
  const Root r = root_state(t, e);
  const float* sd = t.sensordata + (size_t)e * t.nsensordata;
  stage_env(t, e, r, sd, lane, ev);
  const FootVals* F = ev->f;
  // ---- terminations (termination_manager.py:87-97)
  bool tm_v = false;
  {
    const int k = lane;
    bool v = false;
    switch (k < t.ntermination ? t.termination_kind[k] : -1) {
      case MJX_TM_TIME_OUT: v = len >= t.max_episode_length; break;
      case MJX_TM_BAD_ORIENT: v = fabsf(acosf(-r.grav_b.z)) > t.termination_p0[k]; break;  // NaN -> false, as torch
      case MJX_TM_ILLEGAL_CONTACT: v = ev->illegal; break;
      case MJX_TM_ROOT_HEIGHT:  // envs/mdp/terminations.py root_height_below_minimum
        v = t.xpos[((size_t)e * t.nbody + t.root_body) * 3 + 2] < t.termination_p0[k];
        break;
      case MJX_TM_EXCESSIVE_FORCE: {  // tasks/jump/mdp/terminations.py:15-45
        float fmax = 0.f;
        for (int s = 0; s < t.nfeet; s++)
          fmax = fmaxf(fmax, sqrtf(F[s].fx * F[s].fx + F[s].fy * F[s].fy + F[s].fz * F[s].fz));
        v = fmax > t.termination_p0[k];
      } break;
    }
    if (k < t.ntermination) {
      t.term_dones[(size_t)k * t.nworld + e] = v;
      tm_v = v;
    }
  }
  const bool is_to = lane < t.ntermination && t.termination_is_timeout[lane];
  const bool truncated = __ballot(tm_v && is_to) != 0ull;
  const bool terminated = __ballot(tm_v && !is_to) != 0ull;
  const bool reset = terminated || truncated;
  if (lane == 0) {
    t.terminated[e] = terminated;
    t.time_outs[e] = truncated;
    t.reset_buf[e] = reset;
  }
  // ---- rewards (reward_manager.py:77-91)
  const float dt = t.step_dt;
  const int nj = t.njoint;
  // every global value a term reads, loaded before the switch: the wave walks the cases one
  // after another (lane per term), so a load inside a case is a round trip of its own
  // (the twist command is [nworld, 3]; the jump command [nworld, 1], which no term reads)
  float cmd[3] = {0.f, 0.f, 0.f};
  if (t.command_kind == MJX_CMD_TWIST) {
    const float* cmdp = t.command + (size_t)e * 3;
    cmd[0] = cmdp[0]; cmd[1] = cmdp[1]; cmd[2] = cmdp[2];
  }
  float hm[3] = {0.f, 0.f, 0.f};
  if (t.angmom_adr >= 0) { hm[0] = sd[t.angmom_adr]; hm[1] = sd[t.angmom_adr + 1]; hm[2] = sd[t.angmom_adr + 2]; }
  const float selfcol = t.selfcol_found_adr >= 0 ? sd[t.selfcol_found_adr] : 0.f;
  float* es = t.episode_sums + (size_t)(lane < t.nreward ? lane : 0) * t.nworld + e;
  const float es_old = lane < t.nreward ? *es : 0.f;
  float total = 0.f;
  do {
    const int k = lane;
    const float w = k < t.nreward ? t.reward_weight[k] : 0.f;
    float* sr = t.step_reward + (size_t)e * t.nreward + k;
    if (w == 0.f) {
      if (k < t.nreward) *sr = 0.f;
      break;
    }
    const float p0 = t.reward_p0[k], p1 = t.reward_p1[k], p2 = t.reward_p2[k];
    float f = 0.f;
    switch (t.reward_kind[k]) {
      case MJX_RW_TRACK_LIN: {  // rewards.py:23-40
        float dx = cmd[0] - r.lin_b.x, dy = cmd[1] - r.lin_b.y;
        f = expf(-(dx * dx + dy * dy + r.lin_b.z * r.lin_b.z) / (p0 * p0));
      } break;
      case MJX_RW_TRACK_ANG: {  // rewards.py:43-60
        float dz = cmd[2] - r.ang_b.z;
        f = expf(-(dz * dz + r.ang_b.x * r.ang_b.x + r.ang_b.y * r.ang_b.y) / (p0 * p0));
      } break;
      case MJX_RW_FLAT_ORIENT:  // rewards.py:63-85
        f = expf(-(ev->og_x * ev->og_x + ev->og_y * ev->og_y) / (p0 * p0));
        break;
      case MJX_RW_POSE: {  // rewards.py:291-359 (p0 walking, p1 running threshold)
        const float speed = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) + fabsf(cmd[2]);
        const float s = js.pose[speed < p0 ? 0 : (speed < p1 ? 1 : 2)];
        f = expf(-s / (float)nj);
      } break;
      case MJX_RW_BODY_ANG_VEL:  // rewards.py:98-107
        f = ev->ocv0 * ev->ocv0 + ev->ocv1 * ev->ocv1;
        break;
      case MJX_RW_ANGMOM: {  // rewards.py:110-120
        f = hm[0] * hm[0] + hm[1] * hm[1] + hm[2] * hm[2];
        atomicAdd(&acc->metric_sum[MJX_MT_ANGMOM], sqrtf(f));
        atomicAdd(&acc->metric_cnt[MJX_MT_ANGMOM], 1.f);
      } break;
      case MJX_RW_JOINT_POS_LIMITS: f = js.lim; break;  // envs/mdp/rewards.py:73-88
      case MJX_RW_ACTION_RATE: f = js.rate; break;       // envs/mdp/rewards.py:56-60
      case MJX_RW_FEET_AIR_TIME: {  // rewards.py:123-152 (p0 min, p1 max, p2 cmd thr)
        float in_air_t = 0.f, in_air_n = 0.f;
        for (int s = 0; s < t.nfeet; s++) {
          const float at = F[s].air;
          f += (at > p0 && at < p1) ? 1.f : 0.f;
          if (at > 0.f) { in_air_t += at; in_air_n += 1.f; }
        }
        atomicAdd(&acc->metric_sum[MJX_MT_AIR_TIME], in_air_t);
        atomicAdd(&acc->metric_cnt[MJX_MT_AIR_TIME], in_air_n);
        f *= command_gate(t, cmd, p2, 0.f);
      } break;
      case MJX_RW_FEET_CLEARANCE: {  // rewards.py:155-177 (p0 target, p1 cmd thr)
        for (int s = 0; s < t.nfeet; s++)
          f += fabsf(F[s].z - p0) * sqrtf(F[s].vx * F[s].vx + F[s].vy * F[s].vy);
        f *= command_gate(t, cmd, p1, 0.f);
      } break;
      case MJX_RW_FEET_SWING: {  // rewards.py:180-229 (p0 target, p1 cmd thr)
        float land_n = 0.f, land_h = 0.f;
        for (int s = 0; s < t.nfeet; s++) {
          const size_t i = (size_t)e * t.nfeet + s;
          float peak = F[s].peak;
          if (F[s].found == 0.f) peak = fmaxf(peak, F[s].z);
          const float cc = F[s].cc;
          const bool first = cc > 0.f && cc < dt + 1e-8f;
          if (first) {
            float err = peak / p0 - 1.f;
            f += err * err;
            land_n += 1.f;
            land_h += peak;
            peak = 0.f;
          }
          t.peak_heights[i] = peak;
        }
        atomicAdd(&acc->metric_sum[MJX_MT_PEAK_HEIGHT], land_h);
        atomicAdd(&acc->metric_cnt[MJX_MT_PEAK_HEIGHT], land_n);
        f *= command_gate(t, cmd, p1, 0.f);
      } break;
      case MJX_RW_FEET_SLIP: {  // rewards.py:232-259 (p0 cmd thr)
        float vs = 0.f, n = 0.f;
        for (int s = 0; s < t.nfeet; s++) {
          if (!(F[s].found > 0.f)) continue;
          const float v2 = F[s].vx * F[s].vx + F[s].vy * F[s].vy;
          f += v2;
          vs += sqrtf(v2);
          n += 1.f;
        }
        atomicAdd(&acc->metric_sum[MJX_MT_SLIP], vs);
        atomicAdd(&acc->metric_cnt[MJX_MT_SLIP], n);
        f *= command_gate(t, cmd, p0, 0.f);
      } break;
      case MJX_RW_SOFT_LANDING: {  // rewards.py:262-288 (p0 cmd thr)
        float n = 0.f;
        for (int s = 0; s < t.nfeet; s++) {
          const float cc = F[s].cc;
          if (!(cc > 0.f && cc < dt + 1e-8f)) continue;
          f += sqrtf(F[s].fx * F[s].fx + F[s].fy * F[s].fy + F[s].fz * F[s].fz);
          n += 1.f;
        }
        atomicAdd(&acc->metric_sum[MJX_MT_LANDING], f);
        atomicAdd(&acc->metric_cnt[MJX_MT_LANDING], n);
        f *= command_gate(t, cmd, p0, p1);  // p1: command_name None
      } break;
      case MJX_RW_SELF_COLLISION: f = selfcol; break;  // rewards.py:88-95
      // ---- jump task (tasks/jump/mdp/rewards.py; p0 / p1 as noted)
      case MJX_RW_JUMP_HEIGHT: {  // :20-70, p0 target height, p1 std; stateful, never reset
        const float hz = t.xpos[((size_t)e * t.nbody + t.root_body) * 3 + 2];
        float init = t.jump_initialized[e] ? t.jump_initial[e] : hz;
        t.jump_initial[e] = init;
        t.jump_initialized[e] = 1;
        const float peak = fmaxf(t.jump_peak[e], hz);
        t.jump_peak[e] = peak;
        const float jump = peak - init;
        atomicAdd(&acc->metric_sum[MJX_MT_PEAK_JUMP], peak);
        atomicAdd(&acc->metric_cnt[MJX_MT_PEAK_JUMP], 1.f);
        atomicAdd(&acc->metric_sum[MJX_MT_JUMP_HEIGHT], jump);
        atomicAdd(&acc->metric_cnt[MJX_MT_JUMP_HEIGHT], 1.f);
        f = expf(-((jump - p0) * (jump - p0)) / (p1 * p1));
      } break;
      case MJX_RW_EXPLOSIVE_TAKEOFF: {  // :73-108, p0 power threshold
        bool in_contact = false;
        for (int s = 0; s < t.nfeet; s++) in_contact |= F[s].found > 0.f;
        f = in_contact ? fmaxf(js.power - p0, 0.f) / 1000.f : 0.f;
      } break;
      case MJX_RW_SYNC_EXTENSION: f = js.jv_var; break;  // :111-139
      case MJX_RW_VERTICAL_IMPULSE:  // :142-167
        for (int s = 0; s < t.nfeet; s++) f += fmaxf(F[s].fz, 0.f);
        f /= 500.f;
        break;
      case MJX_RW_AIR_TIME_BONUS: {  // :170-204, p0 min air time
        float amin = 1e30f, in_air_t = 0.f, in_air_n = 0.f;
        for (int s = 0; s < t.nfeet; s++) {
          const float at = F[s].air;
          amin = fminf(amin, at);
          if (at > 0.f) { in_air_t += at; in_air_n += 1.f; }
        }
        atomicAdd(&acc->metric_sum[MJX_MT_AIR_TIME], in_air_t);
        atomicAdd(&acc->metric_cnt[MJX_MT_AIR_TIME], in_air_n);
        f = fmaxf(expf((amin - p0) / p0) - 1.f, 0.f);
      } break;
      case MJX_RW_LANDING_BALANCE: {  // :207-270, p0 stability time; stateful, never reset
        bool in_contact = false;
        for (int s = 0; s < t.nfeet; s++) in_contact |= F[s].found > 0.f;
        const bool just_landed = t.was_in_air[e] && in_contact;
        t.was_in_air[e] = !in_contact;
        const bool upright = fabsf(r.grav_b.z + 1.f) < 0.2f;
        const bool low_vel = sqrtf(r.lin_w.x * r.lin_w.x + r.lin_w.y * r.lin_w.y + r.lin_w.z * r.lin_w.z) < 0.5f &&
                             sqrtf(r.ang_w.x * r.ang_w.x + r.ang_w.y * r.ang_w.y + r.ang_w.z * r.ang_w.z) < 0.5f;
        const float tm = just_landed ? 0.f : t.landing_timer[e];
        const float timer = (upright && low_vel && in_contact) ? tm + dt : 0.f;
        t.landing_timer[e] = timer;
        atomicAdd(&acc->metric_sum[MJX_MT_LANDING_SUCCESS], timer > p0 ? 1.f : 0.f);
        atomicAdd(&acc->metric_cnt[MJX_MT_LANDING_SUCCESS], 1.f);
        f = expf(timer / p0) - 1.f;
      } break;
      case MJX_RW_SYMMETRIC_LANDING: {  // :273-316: both feet in first contact
        bool both = t.nfeet >= 2;
        for (int s = 0; s < 2 && s < t.nfeet; s++) {
          const float cc = F[s].cc;
          both = both && cc > 0.f && cc < dt + 1e-8f;
        }
        f = both ? 1.f : 0.f;
      } break;
      case MJX_RW_ACTION_ACC: f = js.acc2; break;        // envs/mdp/rewards.py:63-70
      case MJX_RW_JOINT_TORQUES: f = js.torque2; break;  // envs/mdp/rewards.py:32-37
      case MJX_RW_IS_ALIVE: f = terminated ? 0.f : 1.f; break;  // envs/mdp/rewards.py:22-24
    }
    float v = f * w * dt;
    if (!isfinite(v)) v = 0.f;  // nan_to_num
    total = v;
    const float es_new = es_old + v;
    *sr = v / dt;
    // ---- reset bookkeeping of this step's resets (reward manager log)
    if (reset) {
      atomicAdd(&acc->reward[k], es_new);
      *es = 0.f;
    } else {
      *es = es_new;
    }
  } while (0);
  // reward total in term order (sequential, as the reference's per-term accumulation)
  {
    float tot = 0.f;
    for (int k = 0; k < t.nreward; k++) tot += __shfl(total, k);
    if (lane == 0) t.reward_buf[e] = tot;
  }
  // zero-weight terms still hand their (unchanged) episode sums to the log on reset
  for (int k = lane; k < t.nreward; k += 64) {
    if (reset && t.reward_weight[k] == 0.f) {
      float* es = t.episode_sums + (size_t)k * t.nworld + e;
      atomicAdd(&acc->reward[k], *es);
      *es = 0.f;
    }
  }
  // stored after the env's loads (a store ahead of them would hold up their waits)
  if (lane == 0) t.episode_length[e] = len;
  // ---- reset bookkeeping (termination/command manager logs)
  if (reset) {
    if (lane < t.ntermination && tm_v) atomicAdd(&acc->term[lane], 1.f);
    if (lane == 0) {
      atomicAdd(&acc->count, 1.f);
      atomicAdd(&acc->cmd[0], t.metric_err_xy[e]);
      atomicAdd(&acc->cmd[1], t.metric_err_yaw[e]);
      t.metric_err_xy[e] = 0.f;
      t.metric_err_yaw[e] = 0.f;
    }
  }
}

// Wave per env (kPostEnvs envs per block): the joint sums run lane-parallel, the rest of
// the env's terms on lane 0.  Accumulators: block LDS copy, stored as the block's row of
// `part` (plain stores; k_accum sums the rows).  A global atomic per field and block put
// hundreds of blocks on the same few addresses: ~13 us of the kernel's 42 (G1, 4096 envs).
constexpr int kPostEnvs = 16;
constexpr int kAccN = (int)(sizeof(Acc) / sizeof(float));
static_assert(kAccN <= 128, "k_accum: thread per accumulator field");
// WPE: waves per SIMD the register budget targets.  One 16-wave block per CU fits at the
// kernel's natural 68-70 VGPRs (7 waves / SIMD); batches of more than one block per CU
// (Go1 8,192, jump 16,384 envs) take the 64-VGPR form, two blocks per CU, half the rounds
// (a few spilled registers)
template <int WPE>
__global__ __launch_bounds__(64 * kPostEnvs, WPE) void k_post(const mjxTaskDesc* __restrict__ T,
                                                          float* __restrict__ part) {
  const mjxTaskDesc& t = *T;
  __shared__ Acc sh;
  float* shf = reinterpret_cast<float*>(&sh);
  for (int i = threadIdx.x; i < kAccN; i += blockDim.x) shf[i] = 0.f;
  __syncthreads();
  __shared__ EnvVals ev[kPostEnvs];
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kPostEnvs + (threadIdx.x >> 6);
  if (e < t.nworld) {
    const JointSums js = joint_sums(t, e, lane);
    post_env(t, e, js, lane, &sh, &ev[threadIdx.x >> 6]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kAccN; i += blockDim.x) part[(size_t)blockIdx.x * kAccN + i] = shf[i];
}
// acc += the column sums of k_post's block rows: 8 row chunks x 128 field lanes, each
// summing its chunk with 8 independent loads in flight, then an LDS fold of the chunks
constexpr int kAccChunks = 8;
__global__ __launch_bounds__(128 * kAccChunks) void k_accum(const float* __restrict__ part, int nblock,
                                                            Acc* __restrict__ acc) {
  __shared__ float red[kAccChunks][128];
  const int i = threadIdx.x & 127, c = threadIdx.x >> 7;
  float sum = 0.f;
  if (i < kAccN) {
    const int per = (nblock + kAccChunks - 1) / kAccChunks;
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
    for (int k = 0; k < kAccChunks; k++) tot += red[k][i];
    reinterpret_cast<float*>(acc)[i] += tot;
  }
}

__device__ __forceinline__ void resample_command(const mjxTaskDesc& t, int e, uint64_t step,
                                                 uint32_t base) {
  // CommandTerm._resample + UniformVelocityCommand._resample_command (velocity_command.py:65-95)
  const uint64_t seed = t.seed;
  t.cmd_time_left[e] = uniform(t.resampling_time[0], t.resampling_time[1], urand(seed, e, step, base + 0));
  float* c = t.command + (size_t)e * 3;
  c[0] = uniform(t.lin_vel_x[0], t.lin_vel_x[1], urand(seed, e, step, base + 1));
  c[1] = uniform(t.lin_vel_y[0], t.lin_vel_y[1], urand(seed, e, step, base + 2));
  c[2] = uniform(t.ang_vel_z[0], t.ang_vel_z[1], urand(seed, e, step, base + 3));
  if (t.heading_command) {
    t.heading_target[e] = uniform(t.heading[0], t.heading[1], urand(seed, e, step, base + 4));
    t.is_heading_env[e] = urand(seed, e, step, base + 5) <= t.rel_heading_envs;
  }
  t.is_standing_env[e] = urand(seed, e, step, base + 6) <= t.rel_standing_envs;
  t.command_counter[e] += 1;
}

__global__ void k_reset(const mjxTaskDesc* __restrict__ T) {
  const mjxTaskDesc& t = *T;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= t.nworld || !t.reset_buf[e]) return;
  const uint64_t step = *t.step_counter, seed = t.seed;
  const int nj = t.njoint;
  // scene reset: contact-sensor air time, entity targets (scene.py reset_masked)
  for (int f = 0; f < t.nfeet; f++) {
    const size_t i = (size_t)e * t.nfeet + f;
    t.cur_air[i] = t.last_air[i] = t.cur_contact[i] = t.last_contact[i] = 0.f;
  }
  t.last_time[e] = t.time[e];
  for (int j = 0; j < nj; j++) t.joint_pos_target[(size_t)e * nj + j] = 0.f;
  // Scene.write_data_to_sim after the reset (manager_based_rl_env.py:296-298): ctrl <- the
  // cleared targets, which the masked forward then sees
  for (int k = 0; k < nj; k++) t.ctrl[(size_t)e * t.nu + t.ctrl_of_action[k]] = 0.f;
  // reset_root_state_uniform (events.py:81-120)
  float ps[6], vs[6];
  for (int i = 0; i < 6; i++) {
    ps[i] = uniform(t.reset_pose_range[i][0], t.reset_pose_range[i][1], urand(seed, e, step, D_RESET + i));
    vs[i] = uniform(t.reset_vel_range[i][0], t.reset_vel_range[i][1], urand(seed, e, step, D_RESET + 6 + i));
  }
  float* q = t.qpos + (size_t)e * t.nq + t.free_q_adr;
  const float* o = t.env_origins + (size_t)e * 3;
  const float* rs = t.default_root_state;
  q[0] = rs[0] + ps[0] + o[0];
  q[1] = rs[1] + ps[1] + o[1];
  q[2] = rs[2] + ps[2] + o[2];
  float qe[4];
  quat_euler(ps[3], ps[4], ps[5], qe);
  qmul(rs + 3, qe, q + 3);
  float* v = t.qvel + (size_t)e * t.nv + t.free_v_adr;
  V3 ang_b = qapply_inv(q + 3, V3{rs[10] + vs[3], rs[11] + vs[4], rs[12] + vs[5]});
  v[0] = rs[7] + vs[0]; v[1] = rs[8] + vs[1]; v[2] = rs[9] + vs[2];
  v[3] = ang_b.x; v[4] = ang_b.y; v[5] = ang_b.z;
  // reset_joints_by_offset (events.py:123-160): clamp to soft limits
  for (int j = 0; j < nj; j++) {
    float jp = t.default_joint_pos[j] +
               uniform(t.reset_joint_pos_range[0], t.reset_joint_pos_range[1], urand(seed, e, step, D_RESET + 12 + j));
    jp = fminf(fmaxf(jp, t.soft_lo[j]), t.soft_hi[j]);
    float jv = uniform(t.reset_joint_vel_range[0], t.reset_joint_vel_range[1],
                       urand(seed, e, step, D_RESET + 12 + MJX_TASK_MAX_JOINTS + j));
    t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]] = jp;
    t.qvel[(size_t)e * t.nv + t.joint_v_adr[j]] = jv;
  }
  // action manager reset
  for (int j = 0; j < nj; j++) {
    const size_t i = (size_t)e * nj + j;
    t.action[i] = t.prev_action[i] = t.prev_prev_action[i] = 0.f;
  }
  // command manager reset: counter 0 then resample
  t.command_counter[e] = 0;
  if (t.command_kind == MJX_CMD_TWIST) {
    resample_command(t, e, step, D_CMD_RESET);
  } else {  // JumpCommand._resample_command: the configured target height
    t.cmd_time_left[e] = uniform(t.resampling_time[0], t.resampling_time[1], urand(seed, e, step, D_CMD_RESET));
    t.command[e] = t.jump_target_height;
    t.command_counter[e] += 1;
  }
  // event manager reset: interval timers
  if (t.has_push)
    t.push_time_left[e] = uniform(t.push_interval[0], t.push_interval[1], urand(seed, e, step, D_CMD_RESET + 16));
  t.episode_length[e] = 0;
}

// logs of the previous kernels' reductions (k_post ran to completion before this launch)
__device__ void observe_logs(const mjxTaskDesc& t, Acc* __restrict__ acc) {
  {
    if (acc->count > 0.f) {
      for (int k = 0; k < t.nreward; k++) t.log_reward[k] = acc->reward[k] / acc->count / t.episode_length_s;
      for (int k = 0; k < t.ntermination; k++) t.log_termination[k] = acc->term[k];
      t.log_command[0] = acc->cmd[0] / acc->count;
      t.log_command[1] = acc->cmd[1] / acc->count;
    }
    for (int m = 0; m < MJX_MT_COUNT; m++) {
      t.log_metric[m] = acc->metric_sum[m] / fmaxf(acc->metric_cnt[m], 1.f);
      acc->metric_sum[m] = acc->metric_cnt[m] = 0.f;
    }
    for (int k = 0; k < MJX_TASK_MAX_TERMS; k++) acc->reward[k] = acc->term[k] = 0.f;
    acc->cmd[0] = acc->cmd[1] = 0.f;
    acc->count = 0.f;
  }
}
// env e's command update and interval events, before its observations
__device__ void observe_env(const mjxTaskDesc& t, int e) {
  const uint64_t step = *t.step_counter, seed = t.seed;
  const Root r = root_state(t, e);
  if (t.command_kind == MJX_CMD_JUMP) {
    // JumpCommand.compute (tasks/jump/mdp/commands.py:17-62): metrics["target_height"]
    // filled, timer down (a 1e9 s period never elapses), no command update; no interval
    // events in the jump task
    t.metric_err_xy[e] = t.jump_target_height;
    t.cmd_time_left[e] -= t.step_dt;
    return;
  }
  float* c = t.command + (size_t)e * 3;
  // ---- CommandTerm.compute: metrics, timer, resample, heading control (velocity_command.py)
  const float mcs = t.resampling_time[1] / t.step_dt;
  t.metric_err_xy[e] += sqrtf((c[0] - r.lin_b.x) * (c[0] - r.lin_b.x) + (c[1] - r.lin_b.y) * (c[1] - r.lin_b.y)) / mcs;
  t.metric_err_yaw[e] += fabsf(c[2] - r.ang_b.z) / mcs;
  float tl = t.cmd_time_left[e] - t.step_dt;
  t.cmd_time_left[e] = tl;
  if (tl <= 0.f) resample_command(t, e, step, D_CMD);
  if (t.heading_command) {
    V3 fwd = qapply(r.quat, V3{1.f, 0.f, 0.f});
    const float heading = atan2f(fwd.y, fwd.x);
    const float err = wrap_to_pi(t.heading_target[e] - heading);
    t.heading_error[e] = err;
    if (t.is_heading_env[e])
      c[2] = fminf(fmaxf(t.heading_stiffness * err, t.ang_vel_z[0]), t.ang_vel_z[1]);
  }
  if (t.is_standing_env[e]) c[0] = c[1] = c[2] = 0.f;
  // ---- interval event: push_by_setting_velocity (event_manager.py:124-146, events.py:209-223)
  if (t.has_push) {
    float pt = t.push_time_left[e] - t.step_dt;
    if (pt < 1e-6f) {
      pt = uniform(t.push_interval[0], t.push_interval[1], urand(seed, e, step, D_PUSH));
      float u[6];
      for (int i = 0; i < 6; i++)
        u[i] = uniform(t.push_vel_range[i][0], t.push_vel_range[i][1], urand(seed, e, step, D_PUSH + 1 + i));
      float* v = t.qvel + (size_t)e * t.nv + t.free_v_adr;
      const float* qq = t.qpos + (size_t)e * t.nq + t.free_q_adr + 3;
      V3 ang_b = qapply_inv(qq, V3{r.ang_w.x + u[3], r.ang_w.y + u[4], r.ang_w.z + u[5]});
      v[0] = r.lin_w.x + u[0]; v[1] = r.lin_w.y + u[1]; v[2] = r.lin_w.z + u[2];
      v[3] = ang_b.x; v[4] = ang_b.y; v[5] = ang_b.z;
    }
    t.push_time_left[e] = pt;
  }
}

// ---- observations (observation_manager.py:154-208; velocity_env_cfg.py observation terms),
// thread per (env, critic element) after k_observe has updated commands and pushes.  Policy
// element i is the critic's element i (plus noise draw D_NOISE + i); the critic's extras follow.
// jump layout (tasks/jump/jump_env_cfg.py:61-110): policy = [lin 3, ang 3, gravity 3, jpos,
// jvel, actions, height 1, vertical velocity 1, contact nf, air time nf, command 1]; critic =
// policy terms + [foot height nf, sign*log1p|force| 3nf]
__device__ __forceinline__ void obs_jump(const mjxTaskDesc& t, int e, int i) {
  const int nj = t.njoint, nf = t.nfeet;
  const int nput = 9 + 3 * nj + 2 + 2 * nf + 1;
  const float* sd = t.sensordata + (size_t)e * t.nsensordata;
  float* co = t.obs_critic + (size_t)e * t.ncritic;
  if (i < nput) {
    float val, noise = 0.f;
    if (i < 3) {
      val = sd[t.imu_lin_vel_adr + i]; noise = t.noise_lin_vel;
    } else if (i < 6) {
      val = sd[t.imu_ang_vel_adr + i - 3]; noise = t.noise_ang_vel;
    } else if (i < 9) {
      const V3 g = qapply_inv(t.xquat + ((size_t)e * t.nbody + t.root_body) * 4, V3{0.f, 0.f, -1.f});
      val = i == 6 ? g.x : i == 7 ? g.y : g.z;
      noise = t.noise_gravity;
    } else if (i < 9 + nj) {
      const int j = i - 9;
      val = t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]] - t.default_joint_pos[j];
      noise = t.noise_joint_pos;
    } else if (i < 9 + 2 * nj) {
      val = t.qvel[(size_t)e * t.nv + t.joint_v_adr[i - 9 - nj]]; noise = t.noise_joint_vel;
    } else if (i < 9 + 3 * nj) {
      val = t.action[(size_t)e * nj + i - 9 - 2 * nj];
    } else {
      const int x = i - 9 - 3 * nj;
      if (x == 0) {  // height_above_ground: root z (flat terrain height 0, observations.py:19-41)
        val = t.xpos[((size_t)e * t.nbody + t.root_body) * 3 + 2];
      } else if (x == 1) {  // vertical_velocity: root_link_lin_vel_w z
        val = root_state(t, e).lin_w.z;
      } else if (x < 2 + nf) {
        val = sd[t.feet_found_adr[x - 2]] > 0.f ? 1.f : 0.f;
      } else if (x < 2 + 2 * nf) {
        val = t.cur_air[(size_t)e * nf + x - 2 - nf];
      } else {
        val = t.command[e];
      }
    }
    co[i] = val;
    t.obs_policy[(size_t)e * t.npolicy + i] =
        t.corrupt_policy && noise > 0.f ? val + uniform(-noise, noise, urand(t.seed, e, *t.step_counter, D_NOISE + i)) : val;
    return;
  }
  const int x = i - nput;
  float v;
  if (x < nf) {
    v = t.site_xpos[((size_t)e * t.nsite + t.foot_site[x]) * 3 + 2];
  } else {
    const int y = x - nf, fs = y / 3, k = y % 3;
    const float fv = sd[t.feet_force_adr[fs] + k];
    v = copysignf(log1pf(fabsf(fv)), fv) * (fv != 0.f ? 1.f : 0.f);
  }
  co[i] = v;
}

// observation elements of env e: the critic's (the jump layout, or the velocity layout)
__device__ __forceinline__ int obs_count(const mjxTaskDesc& t) {
  if (t.command_kind == MJX_CMD_JUMP) return t.ncritic;
  const int nput = 9 + 3 * t.njoint + 3;
  return t.critic_extras ? nput + 6 * t.nfeet : nput;
}
__device__ void obs_elem(const mjxTaskDesc& t, int e, int i) {
  if (t.command_kind == MJX_CMD_JUMP) {
    obs_jump(t, e, i);
    return;
  }
  const int nj = t.njoint;
  const int nput = 9 + 3 * nj + 3;  // elements shared by the policy and critic groups
  const float* sd = t.sensordata + (size_t)e * t.nsensordata;
  float* co = t.obs_critic + (size_t)e * t.ncritic;
  if (i < nput) {
    float val, noise = 0.f;
    if (i < 3) {
      val = sd[t.imu_lin_vel_adr + i]; noise = t.noise_lin_vel;
    } else if (i < 6) {
      val = sd[t.imu_ang_vel_adr + i - 3]; noise = t.noise_ang_vel;
    } else if (i < 9) {
      const V3 g = qapply_inv(t.xquat + ((size_t)e * t.nbody + t.root_body) * 4, V3{0.f, 0.f, -1.f});
      val = i == 6 ? g.x : i == 7 ? g.y : g.z;
      noise = t.noise_gravity;
    } else if (i < 9 + nj) {
      const int j = i - 9;
      val = t.qpos[(size_t)e * t.nq + t.joint_q_adr[j]] - t.default_joint_pos[j];
      noise = t.noise_joint_pos;
    } else if (i < 9 + 2 * nj) {
      val = t.qvel[(size_t)e * t.nv + t.joint_v_adr[i - 9 - nj]]; noise = t.noise_joint_vel;
    } else if (i < 9 + 3 * nj) {
      val = t.action[(size_t)e * nj + i - 9 - 2 * nj];
    } else {
      val = t.command[(size_t)e * 3 + i - 9 - 3 * nj];
    }
    co[i] = val;
    const bool noisy = t.corrupt_policy != 0;
    t.obs_policy[(size_t)e * t.npolicy + i] =
        noisy && noise > 0.f ? val + uniform(-noise, noise, urand(t.seed, e, *t.step_counter, D_NOISE + i)) : val;
    return;
  }
  const int x = i - nput, nf = t.nfeet, s = x % nf, blk = x / nf;
  float v;
  if (blk == 0) {
    v = t.site_xpos[((size_t)e * t.nsite + t.foot_site[s]) * 3 + 2];
  } else if (blk == 1) {
    v = t.cur_air[(size_t)e * nf + s];
  } else if (blk == 2) {
    v = sd[t.feet_found_adr[s]] > 0.f ? 1.f : 0.f;
  } else {  // blocks 3..5: foot s's force, 3 components per foot in foot order
    const int y = x - 3 * nf, fs = y / 3, k = y % 3;
    const float fv = sd[t.feet_force_adr[fs] + k];
    v = copysignf(log1pf(fabsf(fv)), fv) * (fv != 0.f ? 1.f : 0.f);
  }
  co[i] = v;
}

// Command update, interval events and observations as one launch, a wave per env: lane 0
// runs the env's command / push update, then the wave's lanes write its observation elements
// (which read the updated command and velocities).  Each env touches only its own state, so
// the wave-level hand-off replaces the launch boundary of two kernels (observe, then
// observations), one dispatch and gap fewer on the env step's critical path.
// Block 0 first folds k_post's block partials into the accumulators (the work of a separate
// k_accum launch, one dispatch and launch gap fewer on the env step's critical path; the
// partials are complete, k_post ran before this launch), then writes the logs.
constexpr int kObsEnvs = 4;
__global__ __launch_bounds__(64 * kObsEnvs, 8) void k_observe_obs(const mjxTaskDesc* __restrict__ T,
                                                               Acc* __restrict__ acc,
                                                               const float* __restrict__ part,
                                                               int nblock) {
  const mjxTaskDesc& t = *T;
  if (blockIdx.x == 0 && nblock > 0) {
    constexpr int kCh = 64 * kObsEnvs / 128;  // row chunks: 128 field lanes each
    __shared__ float red[kCh][128];
    const int i = threadIdx.x & 127, c = threadIdx.x >> 7;
    float sum = 0.f;
    if (i < kAccN) {
      const int per = (nblock + kCh - 1) / kCh;
      const int b0 = c * per, b1 = min(nblock, b0 + per);
      float sv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int b = b0;
      for (; b + 7 < b1; b += 8)
#pragma unroll
        for (int u = 0; u < 8; u++) sv[u] += part[(size_t)(b + u) * kAccN + i];
      for (; b < b1; b++) sv[0] += part[(size_t)b * kAccN + i];
      sum = ((sv[0] + sv[1]) + (sv[2] + sv[3])) + ((sv[4] + sv[5]) + (sv[6] + sv[7]));
    }
    red[c][i] = sum;
    __syncthreads();
    if (c == 0 && i < kAccN) {
      float tot = 0.f;
#pragma unroll
      for (int k = 0; k < kCh; k++) tot += red[k][i];
      reinterpret_cast<float*>(acc)[i] += tot;
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) observe_logs(t, acc);
  const int e = blockIdx.x * kObsEnvs + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (e >= t.nworld) return;
  if (lane == 0) observe_env(t, e);
  // lane 0's stores are complete and visible to the wave's loads (workgroup scope: one CU)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const int nel = obs_count(t);
  for (int i = lane; i < nel; i += 64) obs_elem(t, e, i);
}

// Terrain-level curriculum over the reset mask (tasks/velocity/mdp/curriculums.py:30-64,
// terrains/terrain_importer.py:186-201), thread per env: a resetting env moves one level up
// when it walked more than half a patch from its origin, down when less than half its
// commanded distance over an episode; past the top level it draws a level (counter hash of
// seed, env, counter); its origin becomes the sub-terrain origin [level, type].
__global__ void k_terrain(int nworld, const uint8_t* __restrict__ mask, const float* __restrict__ xpos,
                          int nbody, int root, const float* __restrict__ cmd, float half_patch,
                          float ep_len_s, const int64_t* __restrict__ types, int64_t* __restrict__ levels,
                          const float* __restrict__ torig, int nrows, int ncols,
                          float* __restrict__ origins, uint64_t seed, const uint64_t* __restrict__ counter) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nworld || !mask[e]) return;
  const float* p = xpos + ((size_t)e * nbody + root) * 3;
  float* o = origins + (size_t)e * 3;
  const float dx = p[0] - o[0], dy = p[1] - o[1];
  const float dist = sqrtf(dx * dx + dy * dy);
  const float* c = cmd + (size_t)e * 3;
  const bool up = dist > half_patch;
  const bool down = !up && dist < sqrtf(c[0] * c[0] + c[1] * c[1]) * ep_len_s * 0.5f;
  int64_t lv = levels[e] + (up ? 1 : 0) - (down ? 1 : 0);
  if (lv >= nrows) {
    lv = (int64_t)(urand(seed, (uint32_t)e, *counter, D_TERRAIN) * (float)nrows);
    if (lv >= nrows) lv = nrows - 1;
  } else if (lv < 0) {
    lv = 0;
  }
  levels[e] = lv;
  const int64_t ty = types[e];
  const float* src = torig + ((size_t)lv * ncols + (size_t)ty) * 3;
  o[0] = src[0]; o[1] = src[1]; o[2] = src[2];
}
// mean level (the curriculum's logged state) and the draw counter's advance: one block
__global__ __launch_bounds__(256) void k_terrain_mean(int nworld, const int64_t* __restrict__ levels,
                                                      float* __restrict__ mean, uint64_t* __restrict__ counter) {
  __shared__ float red[256];
  float sum = 0.f;
  for (int e = threadIdx.x; e < nworld; e += 256) sum += (float)levels[e];
  red[threadIdx.x] = sum;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *mean = red[0] / (float)(nworld > 0 ? nworld : 1);
    *counter += 1;
  }
}

}  // namespace mjxt

// ----------------------------------------------------------------------------- C ABI
struct mjxTask_ {
  mjxTaskDesc host;
  mjxTaskDesc* dev = nullptr;
  mjxt::Acc* acc = nullptr;
  float* part = nullptr;  // [nblock][kAccN] k_post block partials
  int nworld = 0;
  // k_post's partials not yet folded into acc (k_observe_obs folds them; a second post before
  // an observe folds the first's with a k_accum launch of its own)
  int pending_nblock = 0;
  int ncu = 256;  // compute units of the device the task was created on
};

static thread_local std::string g_task_err;
static int task_fail(const std::string& s) {
  g_task_err = s;
  return -1;
}

extern "C" {

size_t mjx_task_desc_size(void) { return sizeof(mjxTaskDesc); }

}  // extern "C"

// Every index the kernels dereference, checked against the sizes the descriptor declares, and
// every term / command kind against the buffers and layout it reads, before anything reaches
// the device: a mismatch is an error code and mjx_task_last_error, never an out-of-bounds
// access on the GPU (round 5: a twist-command read on the jump task's [nworld, 1] command
// faulted the device).  Returns "" when the descriptor is consistent.
static std::string validate_task(const mjxTaskDesc& t) {
  auto in = [](int v, int n) { return v >= 0 && v < n; };
  auto span = [](int adr, int len, int n) { return adr >= 0 && adr + len <= n; };
  char buf[256];
  auto err = [&](const char* fmt, int a, int b) {
    snprintf(buf, sizeof buf, fmt, a, b);
    return std::string(buf);
  };
  if (t.nworld <= 0 || t.nq <= 0 || t.nv <= 0 || t.nu <= 0 || t.nbody <= 0 || t.nsensordata < 0 ||
      t.nsite < 0)
    return "non-positive model or batch size";
  if (t.njoint < 1 || t.njoint > MJX_TASK_MAX_JOINTS || t.nfeet < 0 || t.nfeet > MJX_TASK_MAX_FEET ||
      t.nreward < 0 || t.nreward > MJX_TASK_MAX_TERMS || t.ntermination < 0 ||
      t.ntermination > MJX_TASK_MAX_TERMS || t.nillegal < 0 || t.nillegal > MJX_TASK_MAX_CONTACT_SLOTS)
    return "task descriptor exceeds compiled capacities";
  if (t.command_kind != MJX_CMD_TWIST && t.command_kind != MJX_CMD_JUMP)
    return err("unknown command_kind %d (%d kinds)", t.command_kind, 2);
  // buffers every launch reads or writes
  const void* need[] = {t.qpos, t.qvel, t.ctrl, t.time, t.xpos, t.xquat, t.cvel, t.subtree_com,
                        t.sensordata, t.env_origins, t.action, t.prev_action, t.prev_prev_action,
                        t.joint_pos_target, t.episode_length, t.command, t.cmd_time_left,
                        t.command_counter, t.metric_err_xy, t.metric_err_yaw, t.episode_sums,
                        t.step_reward, t.reward_buf, t.reset_buf, t.terminated, t.time_outs,
                        t.term_dones, t.obs_policy, t.obs_critic, t.log_reward, t.log_termination,
                        t.log_command, t.log_metric, t.step_counter};
  for (size_t i = 0; i < sizeof need / sizeof need[0]; i++)
    if (!need[i]) return err("required buffer %d of the descriptor is null", (int)i, 0);
  if (t.nfeet > 0 && (!t.site_xpos || !t.cur_air || !t.last_air || !t.cur_contact ||
                      !t.last_contact || !t.last_time || !t.peak_heights))
    return "feet declared but a foot buffer (site_xpos, air / contact times, peak heights) is null";
  if (t.has_push && !t.push_time_left) return "has_push without push_time_left";
  if (t.command_kind == MJX_CMD_TWIST && !t.is_standing_env)
    return "twist command without is_standing_env";
  if (t.command_kind == MJX_CMD_TWIST && t.heading_command &&
      (!t.heading_target || !t.heading_error || !t.is_heading_env))
    return "heading_command without its heading buffers";
  // entity indexing
  if (!in(t.root_body, t.nbody)) return err("root_body %d outside [0, %d)", t.root_body, t.nbody);
  if (t.orient_body >= t.nbody) return err("orient_body %d outside [-1, %d)", t.orient_body, t.nbody);
  if (!span(t.free_q_adr, 7, t.nq)) return err("free joint qpos %d + 7 past nq %d", t.free_q_adr, t.nq);
  if (!span(t.free_v_adr, 6, t.nv)) return err("free joint qvel %d + 6 past nv %d", t.free_v_adr, t.nv);
  for (int j = 0; j < t.njoint; j++) {
    if (!in(t.joint_q_adr[j], t.nq)) return err("joint %d qpos address outside [0, nq=%d)", j, t.nq);
    if (!in(t.joint_v_adr[j], t.nv)) return err("joint %d qvel address outside [0, nv=%d)", j, t.nv);
    if (!in(t.ctrl_of_action[j], t.nu)) return err("action %d ctrl index outside [0, nu=%d)", j, t.nu);
    if (!in(t.target_of_action[j], t.njoint))
      return err("action %d joint_pos_target column outside [0, njoint=%d)", j, t.njoint);
  }
  for (int s = 0; s < t.nfeet; s++) {
    if (!in(t.foot_site[s], t.nsite)) return err("foot %d site outside [0, nsite=%d)", s, t.nsite);
    if (!in(t.foot_site_body[s], t.nbody)) return err("foot %d body outside [0, nbody=%d)", s, t.nbody);
    if (!in(t.feet_found_adr[s], t.nsensordata))
      return err("foot %d found sensor outside [0, nsensordata=%d)", s, t.nsensordata);
    if (!span(t.feet_force_adr[s], 3, t.nsensordata))
      return err("foot %d force sensor + 3 past nsensordata %d", s, t.nsensordata);
  }
  for (int k = 0; k < t.nillegal; k++)
    if (!in(t.illegal_found_adr[k], t.nsensordata))
      return err("illegal-contact slot %d outside [0, nsensordata=%d)", k, t.nsensordata);
  if (!span(t.imu_lin_vel_adr, 3, t.nsensordata) || !span(t.imu_ang_vel_adr, 3, t.nsensordata))
    return err("imu velocity sensors (%d, %d) + 3 past nsensordata", t.imu_lin_vel_adr, t.imu_ang_vel_adr);
  if (t.angmom_adr >= 0 && !span(t.angmom_adr, 3, t.nsensordata))
    return err("angular-momentum sensor %d + 3 past nsensordata %d", t.angmom_adr, t.nsensordata);
  if (t.selfcol_found_adr >= t.nsensordata)
    return err("self-collision sensor %d outside [-1, %d)", t.selfcol_found_adr, t.nsensordata);
  if (t.max_episode_length <= 0 || !(t.step_dt > 0.f)) return "non-positive episode length or step_dt";
  // terms: kinds, and what each reads
  for (int k = 0; k < t.nreward; k++) {
    const int kind = t.reward_kind[k];
    if (!in(kind, MJX_RW_IS_ALIVE + 1)) return err("reward %d: unknown kind %d", k, kind);
    switch (kind) {
      // read the twist command [nworld, 3] (the feet terms only gate on it, and command_gate
      // passes them ungated under another command kind: the jump task's soft_landing)
      case MJX_RW_TRACK_LIN: case MJX_RW_TRACK_ANG: case MJX_RW_POSE:
        if (t.command_kind != MJX_CMD_TWIST)
          return err("reward %d: kind %d reads the twist command, command_kind is not MJX_CMD_TWIST", k, kind);
        break;
      case MJX_RW_ANGMOM:
        if (t.angmom_adr < 0) return err("reward %d: kind %d needs angmom_adr", k, kind);
        break;
      case MJX_RW_SELF_COLLISION:
        if (t.selfcol_found_adr < 0) return err("reward %d: kind %d needs selfcol_found_adr", k, kind);
        break;
      case MJX_RW_JUMP_HEIGHT:
        if (!t.jump_peak || !t.jump_initial || !t.jump_initialized)
          return err("reward %d: kind %d needs the jump_height state buffers", k, kind);
        break;
      case MJX_RW_LANDING_BALANCE:
        if (!t.landing_timer || !t.was_in_air)
          return err("reward %d: kind %d needs landing_timer / was_in_air", k, kind);
        break;
      default: break;
    }
    if ((kind == MJX_RW_EXPLOSIVE_TAKEOFF || kind == MJX_RW_JOINT_TORQUES || kind == MJX_RW_ACTION_ACC ||
         kind == MJX_RW_SYNC_EXTENSION) && !t.actuator_force)
      return err("reward %d: kind %d reads actuator_force, which is null", k, kind);
  }
  if (t.actuator_force)
    for (int j = 0; j < t.njoint; j++)
      if (!in(t.act_ctrl[j], t.nu)) return err("actuator %d ctrl index outside [0, nu=%d)", j, t.nu);
  for (int k = 0; k < t.ntermination; k++) {
    const int kind = t.termination_kind[k];
    if (!in(kind, MJX_TM_EXCESSIVE_FORCE + 1)) return err("termination %d: unknown kind %d", k, kind);
    if (kind == MJX_TM_ILLEGAL_CONTACT && t.nillegal == 0)
      return err("termination %d: illegal_contact with no contact slots (%d)", k, t.nillegal);
  }
  // observation layouts (k_observe_obs writes exactly these widths)
  const int nj = t.njoint, nf = t.nfeet;
  if (t.command_kind == MJX_CMD_JUMP) {
    if (t.npolicy != 9 + 3 * nj + 3 + 2 * nf || t.ncritic != t.npolicy + 4 * nf)
      return err("observation widths (%d, %d) do not match the jump task layout", t.npolicy, t.ncritic);
  } else {
    const int nput = 9 + 3 * nj + 3;
    if (t.npolicy != nput || t.ncritic != nput + (t.critic_extras ? 6 * nf : 0))
      return err("observation widths (%d, %d) do not match the velocity task layout", t.npolicy, t.ncritic);
    if (t.critic_extras && nf == 0) return "critic_extras with no feet";
  }
  return "";
}

extern "C" {

int mjx_task_create(const mjxTaskDesc* desc, mjxTask** out) {
  if (!desc || !out) return task_fail("null argument");
  if (desc->njoint > MJX_TASK_MAX_JOINTS || desc->nfeet > MJX_TASK_MAX_FEET ||
      desc->nreward > MJX_TASK_MAX_TERMS || desc->ntermination > MJX_TASK_MAX_TERMS ||
      desc->nillegal > MJX_TASK_MAX_CONTACT_SLOTS)
    return task_fail("task descriptor exceeds compiled capacities");
  {
    const std::string why = validate_task(*desc);
    if (!why.empty()) return task_fail("mjx_task_create: " + why);
  }
  auto* t = new mjxTask_();
  t->host = *desc;
  t->nworld = desc->nworld;
  const size_t nblock = ((size_t)t->nworld + mjxt::kPostEnvs - 1) / mjxt::kPostEnvs;
  if (hipMalloc((void**)&t->dev, sizeof(mjxTaskDesc)) != hipSuccess ||
      hipMalloc((void**)&t->acc, sizeof(mjxt::Acc)) != hipSuccess ||
      hipMalloc((void**)&t->part, sizeof(float) * mjxt::kAccN * (nblock > 0 ? nblock : 1)) != hipSuccess) {
    delete t;
    return task_fail("hipMalloc failed");
  }
  {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
      t->ncu = ncu;
  }
  if (hipMemcpy(t->dev, desc, sizeof(mjxTaskDesc), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(t->acc, 0, sizeof(mjxt::Acc)) != hipSuccess) {
    delete t;
    return task_fail("upload failed");
  }
  *out = t;
  return 0;
}

int mjx_task_destroy(mjxTask* t) {
  if (!t) return 0;
  if (t->dev) (void)hipFree(t->dev);
  if (t->acc) (void)hipFree(t->acc);
  if (t->part) (void)hipFree(t->part);
  delete t;
  return 0;
}

#define TASK_LAUNCH(kern, ...)                                                             \
  do {                                                                                     \
    if (!t) return task_fail("null task");                                                 \
    const int nb = (t->nworld + mjxt::kBlock - 1) / mjxt::kBlock;                          \
    hipLaunchKernelGGL(kern, dim3(nb), dim3(mjxt::kBlock), 0, (hipStream_t)stream, __VA_ARGS__); \
    hipError_t e_ = hipGetLastError();                                                      \
    if (e_ != hipSuccess) return task_fail(std::string(#kern ": ") + hipGetErrorString(e_)); \
    return 0;                                                                              \
  } while (0)

int mjx_task_action(mjxTask* t, const float* action, void* stream) {
  if (!t) return task_fail("null task");
  const long n = (long)t->nworld * t->host.njoint;
  hipLaunchKernelGGL(mjxt::k_action, dim3((unsigned)((n + 255) / 256 > 0 ? (n + 255) / 256 : 1)),
                     dim3(256), 0, (hipStream_t)stream, t->dev, action);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : task_fail(std::string("k_action: ") + hipGetErrorString(e));
}
int mjx_task_substep(mjxTask* t, void* stream) { TASK_LAUNCH(mjxt::k_substep, t->dev); }
int mjx_task_post(mjxTask* t, void* stream) {
  if (!t) return task_fail("null task");
  const int nblock = (t->nworld + mjxt::kPostEnvs - 1) / mjxt::kPostEnvs;
  if (t->pending_nblock > 0)  // a post without an observe since: fold its partials first
    hipLaunchKernelGGL(mjxt::k_accum, dim3(1), dim3(128 * mjxt::kAccChunks), 0, (hipStream_t)stream,
                       t->part, t->pending_nblock, t->acc);
  if (nblock > t->ncu)
    hipLaunchKernelGGL(mjxt::k_post<8>, dim3(nblock), dim3(64 * mjxt::kPostEnvs), 0, (hipStream_t)stream,
                       t->dev, t->part);
  else
    hipLaunchKernelGGL(mjxt::k_post<1>, dim3(nblock), dim3(64 * mjxt::kPostEnvs), 0, (hipStream_t)stream,
                       t->dev, t->part);
  t->pending_nblock = nblock;  // folded by the next mjx_task_observe (k_observe_obs block 0)
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : task_fail(std::string("k_post: ") + hipGetErrorString(e));
}
int mjx_task_reset(mjxTask* t, void* stream) { TASK_LAUNCH(mjxt::k_reset, t->dev); }
int mjx_task_observe(mjxTask* t, void* stream) {
  if (!t) return task_fail("null task");
  const int nj = t->host.njoint, nf = t->host.nfeet;
  int nel;
  if (t->host.command_kind == MJX_CMD_JUMP) {
    nel = t->host.ncritic;
    if (t->host.npolicy != 9 + 3 * nj + 3 + 2 * nf || nel != t->host.npolicy + 4 * nf)
      return task_fail("observation sizes do not match the jump task layout");
  } else {
    nel = 9 + 3 * nj + 3 + (t->host.critic_extras ? 6 * nf : 0);
    if (nel > t->host.ncritic || 9 + 3 * nj + 3 > t->host.npolicy)
      return task_fail("observation sizes do not match the velocity task layout");
  }
  (void)nel;
  hipLaunchKernelGGL(mjxt::k_observe_obs, dim3((t->nworld + mjxt::kObsEnvs - 1) / mjxt::kObsEnvs),
                     dim3(64 * mjxt::kObsEnvs), 0, (hipStream_t)stream, t->dev, t->acc, t->part,
                     t->pending_nblock);
  t->pending_nblock = 0;
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : task_fail(std::string("k_observe: ") + hipGetErrorString(e));
}

const char* mjx_task_last_error(void) { return g_task_err.c_str(); }

int mjx_terrain_levels(int nworld, const uint8_t* mask, const float* xpos, int nbody, int root_body,
                       const float* command, float half_patch, float episode_length_s,
                       const int64_t* types, int64_t* levels, const float* terrain_origins,
                       int nrows, int ncols, float* env_origins, uint64_t seed, uint64_t* counter,
                       float* mean_level, void* stream) {
  if (nworld <= 0 || !mask || !xpos || !command || !types || !levels || !terrain_origins ||
      !env_origins || !counter || !mean_level || nrows <= 0 || ncols <= 0 || root_body < 0 ||
      root_body >= nbody)
    return task_fail("mjx_terrain_levels: bad arguments");
  hipLaunchKernelGGL(mjxt::k_terrain, dim3((nworld + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     nworld, mask, xpos, nbody, root_body, command, half_patch, episode_length_s,
                     types, levels, terrain_origins, nrows, ncols, env_origins, seed, counter);
  hipLaunchKernelGGL(mjxt::k_terrain_mean, dim3(1), dim3(256), 0, (hipStream_t)stream, nworld,
                     levels, mean_level, counter);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : task_fail(std::string("k_terrain: ") + hipGetErrorString(e));
}

}  // extern "C"
