/* mjx355_task — fused per-env managers of mjlab's velocity tasks, as HIP kernels.
 *
 * Replaces the torch manager stack of ManagerBasedRlEnv.step()
 * (src/mjlab/envs/manager_based_rl_env.py:272-313) for the velocity task configs
 * (tasks/velocity/velocity_env_cfg.py:33-354, config/{g1,go1}/env_cfgs.py):
 *
 *   mjx_task_action    <- ActionManager.process_action + JointPositionAction.apply_actions
 *                         + Entity.write_data_to_sim (managers/action_manager.py:113-130,
 *                         envs/mdp/actions/joint_actions.py:84-104, entity/data.py:168-180)
 *   mjx_task_substep   <- Scene.update -> ContactSensor._update_air_time_tracking
 *                         (sensor/contact_sensor.py:327-367)
 *   mjx_task_post      <- episode_length += 1, TerminationManager.compute,
 *                         RewardManager.compute, reset bookkeeping of the terminated envs
 *                         (termination_manager.py:87-97, reward_manager.py:77-91, :60-75)
 *   mjx_task_reset     <- the rest of _reset_idx for the masked envs after mj_resetData:
 *                         Scene/sensor reset, reset events (reset_root_state_uniform,
 *                         reset_joints_by_offset), action/command/event manager resets
 *                         (manager_based_rl_env.py:381-416, envs/mdp/events.py:81-206)
 *   mjx_task_observe   <- CommandManager.compute, EventManager.apply("interval"),
 *                         ObservationManager.compute (command_manager.py:53-67,
 *                         velocity_command.py:51-107, event_manager.py:124-146,
 *                         observation_manager.py:154-208)
 *
 * All buffers are device pointers owned by the caller (the torch tensors of the managers
 * and the mjx355 data arena); nothing is copied.  One thread per env; every call is
 * enqueued on `stream` and never synchronises.  Randoms come from a counter-based hash of
 * (seed, env, env-step counter, draw id) — statistically the reference's distributions,
 * not its Philox streams.
 */
#ifndef MJX355_TASK_H_
#define MJX355_TASK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MJX_TASK_MAX_JOINTS 64
#define MJX_TASK_MAX_FEET 8
#define MJX_TASK_MAX_TERMS 24
#define MJX_TASK_MAX_CONTACT_SLOTS 32

/* reward term kinds (tasks/velocity/mdp/rewards.py, envs/mdp/rewards.py) */
enum { MJX_RW_TRACK_LIN = 0, MJX_RW_TRACK_ANG = 1, MJX_RW_FLAT_ORIENT = 2, MJX_RW_POSE = 3,
       MJX_RW_BODY_ANG_VEL = 4, MJX_RW_ANGMOM = 5, MJX_RW_JOINT_POS_LIMITS = 6,
       MJX_RW_ACTION_RATE = 7, MJX_RW_FEET_AIR_TIME = 8, MJX_RW_FEET_CLEARANCE = 9,
       MJX_RW_FEET_SWING = 10, MJX_RW_FEET_SLIP = 11, MJX_RW_SOFT_LANDING = 12,
       MJX_RW_SELF_COLLISION = 13 };
/* termination kinds (envs/mdp/terminations.py, tasks/velocity/mdp/terminations.py) */
enum { MJX_TM_TIME_OUT = 0, MJX_TM_BAD_ORIENT = 1, MJX_TM_ILLEGAL_CONTACT = 2 };
/* global per-step metric slots written by reward terms ("Metrics/<name>_mean") */
enum { MJX_MT_ANGMOM = 0, MJX_MT_AIR_TIME = 1, MJX_MT_PEAK_HEIGHT = 2, MJX_MT_SLIP = 3,
       MJX_MT_LANDING = 4, MJX_MT_COUNT = 5 };

typedef struct mjxTaskDesc_ {
  int nworld, nq, nv, nu, nsensordata, nbody, nsite;
  /* ---- simulation data (mjx355 arena, [nworld, ...]) */
  float *qpos, *qvel, *ctrl, *time;
  const float *xpos, *xquat, *cvel, *subtree_com, *site_xpos, *sensordata;
  /* ---- entity indexing */
  int root_body, free_q_adr, free_v_adr;
  int njoint;                              /* actuated hinge joints = action dim */
  int joint_q_adr[MJX_TASK_MAX_JOINTS], joint_v_adr[MJX_TASK_MAX_JOINTS];
  int ctrl_of_action[MJX_TASK_MAX_JOINTS]; /* action k drives ctrl[ctrl_of_action[k]] */
  int target_of_action[MJX_TASK_MAX_JOINTS]; /* ... and joint_pos_target[:, target_of_action[k]] */
  float action_scale[MJX_TASK_MAX_JOINTS], action_offset[MJX_TASK_MAX_JOINTS];
  float default_joint_pos[MJX_TASK_MAX_JOINTS];
  float soft_lo[MJX_TASK_MAX_JOINTS], soft_hi[MJX_TASK_MAX_JOINTS];
  float std_standing[MJX_TASK_MAX_JOINTS], std_walking[MJX_TASK_MAX_JOINTS],
      std_running[MJX_TASK_MAX_JOINTS];
  float default_root_state[13];            /* pos, quat, lin vel (world), ang vel (world) */
  const float* env_origins;                /* [nworld, 3] */
  int nfeet, foot_site[MJX_TASK_MAX_FEET], foot_site_body[MJX_TASK_MAX_FEET];
  int feet_found_adr[MJX_TASK_MAX_FEET], feet_force_adr[MJX_TASK_MAX_FEET];
  int imu_lin_vel_adr, imu_ang_vel_adr, angmom_adr, selfcol_found_adr;
  int nillegal, illegal_found_adr[MJX_TASK_MAX_CONTACT_SLOTS];
  int orient_body;                         /* body of flat_orientation / body_ang_vel */
  /* ---- timing */
  float step_dt, episode_length_s;
  int max_episode_length;
  /* ---- terms */
  int nreward, reward_kind[MJX_TASK_MAX_TERMS];
  float reward_weight[MJX_TASK_MAX_TERMS], reward_p0[MJX_TASK_MAX_TERMS],
      reward_p1[MJX_TASK_MAX_TERMS], reward_p2[MJX_TASK_MAX_TERMS];
  int ntermination, termination_kind[MJX_TASK_MAX_TERMS], termination_is_timeout[MJX_TASK_MAX_TERMS];
  float termination_p0[MJX_TASK_MAX_TERMS];
  /* ---- command (UniformVelocityCommandCfg) */
  float lin_vel_x[2], lin_vel_y[2], ang_vel_z[2], heading[2], resampling_time[2];
  float rel_standing_envs, rel_heading_envs, heading_stiffness;
  int heading_command;
  /* ---- events */
  float reset_pose_range[6][2];            /* x y z roll pitch yaw */
  float reset_vel_range[6][2];
  float reset_joint_pos_range[2], reset_joint_vel_range[2];
  int has_push;
  float push_interval[2], push_vel_range[6][2];
  /* ---- observations: policy [nworld, npolicy], critic [nworld, ncritic] */
  int npolicy, ncritic, critic_extras;     /* critic = policy terms (+ foot terms if extras) */
  float noise_lin_vel, noise_ang_vel, noise_gravity, noise_joint_pos, noise_joint_vel;
  int corrupt_policy;
  uint64_t seed;
  /* ---- manager state (torch tensors) */
  float *action, *prev_action, *prev_prev_action, *joint_pos_target;  /* [nworld, njoint] */
  int64_t* episode_length;                 /* [nworld] */
  float *command, *heading_target, *heading_error, *cmd_time_left;    /* command [nworld,3] */
  uint8_t *is_heading_env, *is_standing_env;
  int64_t* command_counter;
  float *metric_err_xy, *metric_err_yaw, *push_time_left;
  float* episode_sums;                     /* [nreward, nworld] */
  float *step_reward, *reward_buf;         /* [nworld, nreward], [nworld] */
  uint8_t *reset_buf, *terminated, *time_outs, *term_dones; /* term_dones [ntermination, nworld] */
  float *cur_air, *last_air, *cur_contact, *last_contact, *last_time; /* air time [nworld,nfeet] */
  float* peak_heights;                     /* [nworld, nfeet] */
  float *obs_policy, *obs_critic;
  /* ---- logs (device): per-term episode means, termination counts, command metrics,
   *      global metric means; written when some env resets (or every step for metrics) */
  float* log_reward;                       /* [nreward] */
  float* log_termination;                  /* [ntermination] */
  float* log_command;                      /* [2] error_vel_xy, error_vel_yaw */
  float* log_metric;                       /* [MJX_MT_COUNT] */
  uint64_t* step_counter;                  /* [1] env-step counter for the RNG */
} mjxTaskDesc;

typedef struct mjxTask_ mjxTask;

int mjx_task_create(const mjxTaskDesc* desc, mjxTask** out);
int mjx_task_destroy(mjxTask* task);
int mjx_task_action(mjxTask* task, const float* action, void* stream);
int mjx_task_substep(mjxTask* task, void* stream);
/* writes reset_buf (also usable as the uint8 mask of mjx_reset / mjx_forward_masked) */
int mjx_task_post(mjxTask* task, void* stream);
int mjx_task_reset(mjxTask* task, void* stream);
int mjx_task_observe(mjxTask* task, void* stream);
size_t mjx_task_desc_size(void);  /* sizeof(mjxTaskDesc): ABI check for FFI bindings */
const char* mjx_task_last_error(void);

/* out[i] = q1[i] * q2[i] (wxyz Hamilton product) for n contiguous quaternions, in the
 * reference's 8-multiply operation order without FP contraction: bit-identical to its
 * torch quat_mul (src/mjlab/utils/lab_api/math.py:526-563) in eager mode.  Pointers are
 * device memory, 16-byte aligned.  Returns 0, -1 bad arguments, -2 misaligned, -3 launch. */
int mjx_quat_mul(const float* q1, const float* q2, float* out, long n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MJX355_TASK_H_ */
