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
 * The same kernels run the jump task (command_kind MJX_CMD_JUMP: JumpCommand,
 * tasks/jump/mdp/commands.py:17-62; its reward / termination kinds and observation layout,
 * tasks/jump/jump_env_cfg.py:36-354, including the stateful jump_height_reward and
 * landing_balance terms, which the reference never resets).
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
       MJX_RW_SELF_COLLISION = 13,
       /* jump task (tasks/jump/mdp/rewards.py:20-316, envs/mdp/rewards.py) */
       MJX_RW_JUMP_HEIGHT = 14, MJX_RW_EXPLOSIVE_TAKEOFF = 15, MJX_RW_SYNC_EXTENSION = 16,
       MJX_RW_VERTICAL_IMPULSE = 17, MJX_RW_AIR_TIME_BONUS = 18, MJX_RW_LANDING_BALANCE = 19,
       MJX_RW_SYMMETRIC_LANDING = 20, MJX_RW_ACTION_ACC = 21, MJX_RW_JOINT_TORQUES = 22,
       MJX_RW_IS_ALIVE = 23 };
/* termination kinds (envs/mdp/terminations.py, tasks/velocity/mdp/terminations.py) */
enum { MJX_TM_TIME_OUT = 0, MJX_TM_BAD_ORIENT = 1, MJX_TM_ILLEGAL_CONTACT = 2,
       MJX_TM_ROOT_HEIGHT = 3 /* root_height_below_minimum */,
       MJX_TM_EXCESSIVE_FORCE = 4 /* jump excessive_landing_force */ };
/* global per-step metric slots written by reward terms ("Metrics/<name>_mean") */
enum { MJX_MT_ANGMOM = 0, MJX_MT_AIR_TIME = 1, MJX_MT_PEAK_HEIGHT = 2, MJX_MT_SLIP = 3,
       MJX_MT_LANDING = 4, MJX_MT_PEAK_JUMP = 5, MJX_MT_JUMP_HEIGHT = 6,
       MJX_MT_LANDING_SUCCESS = 7, MJX_MT_COUNT = 8 };
/* command / observation layouts of the fused step */
enum { MJX_CMD_TWIST = 0 /* UniformVelocityCommand */, MJX_CMD_JUMP = 1 /* JumpCommand */ };

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
  /* ---- jump task (Mjlab-Jump-Flat-Unitree-G1, tasks/jump/jump_env_cfg.py:36-354) */
  int command_kind;                        /* MJX_CMD_*: also selects the observation layout */
  float jump_target_height;                /* JumpCommandCfg.target_height (curriculum) */
  const float* actuator_force;             /* [nworld, nu] */
  int act_ctrl[MJX_TASK_MAX_JOINTS];       /* entity actuator i -> ctrl index (actuator order) */
  uint64_t explosive_joints;               /* explosive_takeoff joint selection (bit per joint) */
  float *jump_peak, *jump_initial;         /* jump_height_reward state [nworld] */
  uint8_t* jump_initialized;
  float* landing_timer;                    /* landing_balance state [nworld] */
  uint8_t* was_in_air;
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

/* Terrain-level curriculum of the rough velocity tasks over a reset mask, replacing
 * tasks/velocity/mdp/curriculums.py:30-64 (terrain_levels_vel) + terrains/terrain_importer.py:
 * 186-201 (update_env_origins) for the resetting envs: root xy (xpos[world, root_body]) vs
 * env origin, commanded xy speed x episode length; levels [nworld] int64 updated, env_origins
 * [nworld, 3] set from terrain_origins [nrows, ncols, 3] at (level, type); a level past the
 * top draws uniformly (counter-based hash of seed, env, *counter -- not torch's generator);
 * mean_level = mean of levels; *counter advances by one.  Two launches on `stream`. */
int mjx_terrain_levels(int nworld, const uint8_t* mask, const float* xpos, int nbody, int root_body,
                       const float* command, float half_patch, float episode_length_s,
                       const int64_t* types, int64_t* levels, const float* terrain_origins,
                       int nrows, int ncols, float* env_origins, uint64_t seed, uint64_t* counter,
                       float* mean_level, void* stream);

/* ------------------------------------------------------------------------------------
 * Motion tracking (Mjlab-Tracking-Flat-Unitree-G1): the same fused pattern for the
 * tracking MDP (tasks/tracking/tracking_env_cfg.py:42-317, tasks/tracking/mdp/{commands,rewards,terminations,observations}.py):
 *
 *   mjx_track_action   <- process_action + apply_actions with the encoder bias
 *                         (joint_actions.py:84-104, entity/entity.py:653-670)
 *   mjx_track_post     <- episode_length += 1, TerminationManager.compute (time_out,
 *                         bad_anchor_pos_z_only, bad_anchor_ori, bad_motion_body_pos_z_only),
 *                         RewardManager.compute (6 exp-kernel tracking terms, action_rate_l2,
 *                         joint_pos_limits, self_collision_cost), reset bookkeeping
 *                         (tracking/mdp/terminations.py:18-86, rewards.py:26-120)
 *   mjx_track_reset    <- _reset_idx for the masked envs after mj_resetData: action /
 *                         reward / command / event manager resets; the command reset is
 *                         MotionCommand._resample_command: adaptive failure-binned start
 *                         sampling + reference-state initialisation (commands.py:258-375)
 *   mjx_track_observe  <- CommandManager.compute (MotionCommand._update_metrics,
 *                         _update_command: time step, resampling at the motion end, yaw-
 *                         aligned relative body targets, adaptive-sampling update),
 *                         EventManager.apply("interval") (push), ObservationManager.compute
 *                         (policy 160 / critic 286; tracking/mdp/observations.py:18-69)
 *
 * Motion arrays follow the reference's MotionLoader (commands.py:32-68), indexed by the
 * command's body list.  Randoms: the counter-based hash of mjx_task_*; the multinomial
 * over failure bins is an inverse-CDF draw from the same probabilities.
 * ------------------------------------------------------------------------------------ */
#define MJX_TRACK_MAX_BODIES 32
#define MJX_TRACK_MAX_BINS 1024
#define MJX_TRACK_NMETRIC 13
/* reward kinds (tasks/tracking/mdp/rewards.py, envs/mdp/rewards.py) */
enum { MJX_TR_ANCHOR_POS = 0, MJX_TR_ANCHOR_ORI = 1, MJX_TR_BODY_POS = 2, MJX_TR_BODY_ORI = 3,
       MJX_TR_BODY_LIN_VEL = 4, MJX_TR_BODY_ANG_VEL = 5, MJX_TR_ACTION_RATE = 6,
       MJX_TR_JOINT_LIMIT = 7, MJX_TR_SELF_COLLISION = 8 };
/* termination kinds (tasks/tracking/mdp/terminations.py, envs/mdp/terminations.py) */
enum { MJX_TT_TIME_OUT = 0, MJX_TT_ANCHOR_POS_Z = 1, MJX_TT_ANCHOR_ORI = 2, MJX_TT_BODY_POS_Z = 3,
       MJX_TT_ANCHOR_POS = 4, MJX_TT_BODY_POS = 5 };
/* observation layout: policy = [command anchor_pos? anchor_ori lin_vel? ang_vel jpos(biased)
 * jvel actions], critic = [command anchor_pos anchor_ori body_pos body_ori lin_vel ang_vel
 * jpos jvel actions] (tracking_env_cfg.py:60-110) */

typedef struct mjxTrackDesc_ {
  int nworld, nq, nv, nu, nsensordata, nbody;
  float *qpos, *qvel, *ctrl;
  const float *xpos, *xquat, *cvel, *subtree_com, *sensordata;
  int root_body, free_q_adr, free_v_adr, njoint;
  int joint_q_adr[MJX_TASK_MAX_JOINTS], joint_v_adr[MJX_TASK_MAX_JOINTS];
  int ctrl_of_action[MJX_TASK_MAX_JOINTS], target_of_action[MJX_TASK_MAX_JOINTS];
  float action_scale[MJX_TASK_MAX_JOINTS], action_offset[MJX_TASK_MAX_JOINTS];
  float default_joint_pos[MJX_TASK_MAX_JOINTS];
  float soft_lo[MJX_TASK_MAX_JOINTS], soft_hi[MJX_TASK_MAX_JOINTS];
  const float* encoder_bias;               /* [nworld, njoint] */
  const float* env_origins;                /* [nworld, 3] */
  /* ---- motion (MotionLoader, body-indexed by the command's body list) */
  int nframe, nmb;                         /* motion frames T, command bodies */
  const float *m_joint_pos, *m_joint_vel;  /* [T, njoint] */
  const float *m_body_pos, *m_body_quat, *m_body_lin, *m_body_ang; /* [T, nmb, 3|4] */
  int robot_body[MJX_TRACK_MAX_BODIES];    /* model body of command body k */
  int anchor_motion, anchor_body;          /* command index / model body of the anchor */
  /* ---- timing */
  float step_dt, episode_length_s;
  int max_episode_length;
  /* ---- terms (body terms use bit k of *_bodies for command body k) */
  int nreward, reward_kind[MJX_TASK_MAX_TERMS];
  float reward_weight[MJX_TASK_MAX_TERMS], reward_std[MJX_TASK_MAX_TERMS];
  uint32_t reward_bodies[MJX_TASK_MAX_TERMS];
  int ntermination, termination_kind[MJX_TASK_MAX_TERMS], termination_is_timeout[MJX_TASK_MAX_TERMS];
  float termination_threshold[MJX_TASK_MAX_TERMS];
  uint32_t termination_bodies[MJX_TASK_MAX_TERMS];
  int selfcol_found_adr, imu_lin_vel_adr, imu_ang_vel_adr;
  /* ---- command (MotionCommandCfg) */
  float pose_range[6][2], vel_range[6][2], joint_position_range[2];
  int sampling_mode;                       /* 0 start, 1 uniform, 2 adaptive */
  int bin_count, kernel_size;
  float kernel[8], uniform_ratio, adaptive_alpha;
  /* ---- events */
  int has_push;
  float push_interval[2], push_vel_range[6][2];
  /* ---- observations */
  int npolicy, ncritic, corrupt_policy, policy_anchor_pos, policy_lin_vel;
  float noise_anchor_pos, noise_anchor_ori, noise_lin_vel, noise_ang_vel, noise_joint_pos,
      noise_joint_vel;
  uint64_t seed;
  /* ---- manager state (torch tensors) */
  float *action, *prev_action, *prev_prev_action, *joint_pos_target; /* [nworld, njoint] */
  int64_t* episode_length;
  int64_t* time_steps;                     /* [nworld] motion frame per env */
  float *body_pos_rel, *body_quat_rel;     /* [nworld, nmb, 3|4] relative body targets */
  float *bin_failed_count, *current_bin_failed; /* [bin_count] */
  float* sampling;                         /* [bin_count + 4] scratch: cdf, entropy, top1 */
  float* metrics;                          /* [MJX_TRACK_NMETRIC, nworld] metric tensors */
  float* time_left;
  int64_t* command_counter;
  float* push_time_left;
  float* episode_sums;                     /* [nreward, nworld] */
  float *step_reward, *reward_buf;
  uint8_t *reset_buf, *terminated, *time_outs, *term_dones, *resample_mask;
  float *obs_policy, *obs_critic;
  float *log_reward, *log_termination, *log_metric; /* [nreward] [ntermination] [NMETRIC] */
  uint64_t* step_counter;
} mjxTrackDesc;

typedef struct mjxTrack_ mjxTrack;
int mjx_track_create(const mjxTrackDesc* desc, mjxTrack** out);
int mjx_track_destroy(mjxTrack* task);
int mjx_track_action(mjxTrack* task, const float* action, void* stream);
int mjx_track_post(mjxTrack* task, void* stream);     /* writes reset_buf */
int mjx_track_reset(mjxTrack* task, void* stream);
int mjx_track_observe(mjxTrack* task, void* stream);
size_t mjx_track_desc_size(void);
const char* mjx_track_last_error(void);

/* out[i] = q1[i] * q2[i] (wxyz Hamilton product) for n contiguous quaternions, in the
 * reference's 8-multiply operation order without FP contraction: bit-identical to its
 * torch quat_mul (src/mjlab/utils/lab_api/math.py:526-563) in eager mode.  Pointers are
 * device memory, 16-byte aligned.  Returns 0, -1 bad arguments, -2 misaligned, -3 launch. */
int mjx_quat_mul(const float* q1, const float* q2, float* out, long n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MJX355_TASK_H_ */
