/* mjx355 — MI355X-native batched MuJoCo step: the C ABI of the drop-in boundary.
 *
 * This header is the seam that replaces the reference's physics boundary
 * `mjlab.sim.Simulation` (src/mjlab/sim/sim.py:100-286) and the MuJoCo-Warp calls
 * behind it:
 *
 *   mjx_model_create   <- mujoco_warp.put_model(mj_model)            sim/sim.py:139
 *   mjx_sim_create     <- mujoco_warp.put_data(..., nworld, nconmax,  sim/sim.py:143-149
 *                         njmax) + create_graph()                     sim/sim.py:164-191
 *   mjx_step           <- mujoco_warp.step / wp.capture_launch        sim/sim.py:267-273
 *   mjx_forward        <- mujoco_warp.forward                         sim/sim.py:260-265
 *   mjx_reset          <- mujoco_warp.reset_data(reset=mask)          sim/sim.py:275-286
 *   mjx_field          <- WarpBridge.__getattr__ -> wp.to_torch       sim/sim_data.py:177-240
 *                         (here: a DLPack DLManagedTensor aliasing device memory)
 *   mjx_expand_field   <- expand_model_fields / repeat_array_kernel   sim/sim.py:226-240,
 *                                                                     sim/randomization.py:9-54
 *
 * Conventions: plain C, no exceptions cross the ABI, every call returns an int status
 * (0 = ok) and `mjx_last_error()` gives the message of the last failure on this thread.
 * All device work is enqueued on the HIP stream passed in (`void*` = hipStream_t, NULL =
 * legacy default stream); nothing in step/forward/reset synchronises the host.
 */
#ifndef MJX355_H_
#define MJX355_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MJX_ABI_VERSION 4

/* geom types (MuJoCo mjtGeom numbering) */
enum { MJX_GEOM_PLANE = 0, MJX_GEOM_HFIELD = 1, MJX_GEOM_SPHERE = 2, MJX_GEOM_CAPSULE = 3,
       MJX_GEOM_ELLIPSOID = 4, MJX_GEOM_CYLINDER = 5, MJX_GEOM_BOX = 6, MJX_GEOM_MESH = 7 };
/* joint types (mjtJoint) */
enum { MJX_JNT_FREE = 0, MJX_JNT_BALL = 1, MJX_JNT_SLIDE = 2, MJX_JNT_HINGE = 3 };
/* sensor types (subset of mjtSensor used by mjlab tasks) */
enum { MJX_SENS_GYRO = 0, MJX_SENS_VELOCIMETER = 1, MJX_SENS_ACCELEROMETER = 2,
       MJX_SENS_SUBTREEANGMOM = 3, MJX_SENS_CONTACT = 4, MJX_SENS_FRAMEPOS = 5,
       MJX_SENS_FRAMEQUAT = 6, MJX_SENS_JOINTPOS = 7, MJX_SENS_JOINTVEL = 8 };
/* object types for sensors */
enum { MJX_OBJ_NONE = 0, MJX_OBJ_BODY = 1, MJX_OBJ_XBODY = 2, MJX_OBJ_JOINT = 3,
       MJX_OBJ_GEOM = 5, MJX_OBJ_SITE = 6 };
/* contact sensor reduce modes (sensor/contact_sensor.py:39-44) */
enum { MJX_REDUCE_NONE = 0, MJX_REDUCE_MINDIST = 1, MJX_REDUCE_MAXFORCE = 2,
       MJX_REDUCE_NETFORCE = 3 };
enum { MJX_INT_EULER = 0, MJX_INT_IMPLICITFAST = 1 };

/* Host-side compiled model (fp64 / int32).  Field names follow mjModel.  Array
 * widths per element are in the trailing comment.  Filled by the Python scene
 * compiler (mjlab-1_amd/mjlab_amd/compiler/model.py); consumed by mjx_model_create
 * (uploaded to HBM as fp32) and by the CPU oracle (oracle/oracle.c, fp64). */
typedef struct mjxModelDesc_ {
  int abi_version;
  int nq, nv, nu, nbody, njnt, ngeom, nsite, nsensor, nsensordata, npair;
  int nhfield, nhfielddata, nlevel;
  int nmaskword; /* 32-bit words per contact-sensor geom mask: ceil(ngeom / 32) */
  int iterations, ls_iterations, integrator, cone;
  /* contact sensors: matches per sensor and world considered, the first contact_maxmatch in
   * contact order (>= 1; SimulationCfg.contact_sensor_maxmatch, sim/sim.py:95,141) */
  int contact_maxmatch;
  double timestep, tolerance, ls_tolerance, impratio, meaninertia;
  double gravity[3];
  /* bodies */
  const int32_t *body_parentid, *body_rootid, *body_weldid, *body_jntnum, *body_jntadr,
      *body_dofnum, *body_dofadr, *body_level, *body_childadr /* nbody+1 */,
      *body_child /* >=1 */, *body_mocapid;
  const double *body_pos /*3*/, *body_quat /*4*/, *body_ipos /*3*/, *body_iquat /*4*/,
      *body_mass, *body_inertia /*3*/, *body_subtreemass, *body_invweight0 /*2*/;
  const int32_t *level_start /* nlevel+1 */, *level_body /* nbody */;
  /* joints */
  const int32_t *jnt_type, *jnt_qposadr, *jnt_dofadr, *jnt_bodyid, *jnt_limited;
  const double *jnt_pos /*3*/, *jnt_axis /*3*/, *jnt_range /*2*/, *jnt_solref /*2*/,
      *jnt_solimp /*5*/, *jnt_margin, *jnt_stiffness;
  const double *qpos0 /* nq */, *qpos_spring /* nq */;
  /* dofs */
  const int32_t *dof_bodyid, *dof_jntid, *dof_parentid;
  const uint64_t *dof_bodymask; /* bit b set: dof is on the kinematic chain of body b */
  const double *dof_armature, *dof_damping, *dof_invweight0, *dof_frictionloss;
  /* geoms */
  const int32_t *geom_type, *geom_bodyid, *geom_contype, *geom_conaffinity, *geom_condim,
      *geom_priority, *geom_dataid;
  const double *geom_size /*3*/, *geom_pos /*3*/, *geom_quat /*4*/, *geom_friction /*3*/,
      *geom_solmix, *geom_solref /*2*/, *geom_solimp /*5*/, *geom_margin, *geom_gap,
      *geom_rbound;
  /* sites */
  const int32_t *site_bodyid;
  const double *site_pos /*3*/, *site_quat /*4*/;
  /* actuators (joint transmission, gain fixed, bias affine: <position>/<motor>) */
  const int32_t *actuator_trnid, *actuator_forcelimited, *actuator_ctrllimited;
  const double *actuator_gear, *actuator_gainprm /*3*/, *actuator_biasprm /*3*/,
      *actuator_forcerange /*2*/, *actuator_ctrlrange /*2*/;
  /* sensors */
  const int32_t *sensor_type, *sensor_objtype, *sensor_objid, *sensor_reftype, *sensor_refid,
      *sensor_adr, *sensor_dim, *sensor_intprm /*3*/;
  const uint32_t *sensor_geommask1 /*nmaskword*/, *sensor_geommask2 /*nmaskword*/;
  /* static broadphase: candidate geom pairs, geom1 has the lower geom type.  Pairs with a
   * static terrain geom (a heightfield, or a box on a body welded to the world) come last,
   * grouped by that geom: the engine culls them per geom block (terrain broadphase). */
  const int32_t *pair_geom1, *pair_geom2;
  /* heightfields */
  const int32_t *hfield_nrow, *hfield_ncol, *hfield_adr;
  const double *hfield_size /*4*/, *hfield_data /* nhfielddata, normalised [0,1] */;
} mjxModelDesc;

size_t mjx_model_desc_size(void); /* sizeof(mjxModelDesc): ABI check for FFI bindings */

typedef struct mjxModel_ mjxModel; /* device-resident fp32 model (opaque) */
typedef struct mjxSim_ mjxSim;     /* nworld batched data + workspace (opaque) */

const char* mjx_last_error(void);
int mjx_abi_version(void);

/* Upload a compiled model to HBM (fp32).  `device` = HIP device ordinal. */
int mjx_model_create(const mjxModelDesc* desc, int device, mjxModel** out);
int mjx_model_destroy(mjxModel* model);

/* Allocate batched data for `nworld` worlds.  nconmax: contacts per world (the
 * reference's per-world budget, sim/sim.py:82-92); njmax: constraint rows per world.
 * Data starts at qpos0 (mj_resetData semantics). */
int mjx_sim_create(const mjxModel* model, int nworld, int nconmax, int njmax, mjxSim** out);
/* The same with a max capacity (nconmax <= 64, nconmax <= nconmax_max <= 512, njmax <=
 * njmax_max, and njmax_max >= nconmax_max past 64 contacts: every contact makes a row, so the
 * reference's njmax bounds a world's contacts too): the step
 * runs at (nconmax, njmax) per world -- the fast LDS carve -- and a world whose contacts or
 * rows overflow it in a substep is re-solved at (nconmax_max, njmax_max) instead of
 * truncated (the reference's budget semantics: its nconmax is pooled, sim/sim.py:82-92; its
 * njmax, 300 rows for the velocity tasks, bounds each world).  Only what overflows the max
 * capacity is dropped (counted by mjx_sim_stats).  The contact output arrays hold
 * nconmax_max slots per world; a masked forward re-solves its overflowing worlds too.  A batch
 * the engine splits into concurrent halves (large batches of models without Newton row
 * classes) re-solves behind each half's launches; only a split forced onto a model with row
 * classes (MJX355_SPLIT, diagnostic) keeps the fast carve as its max capacity (mjx_sim_info
 * reports the capacity wired). */
int mjx_sim_create_ex(const mjxModel* model, int nworld, int nconmax, int njmax, int nconmax_max,
                      int njmax_max, mjxSim** out);
int mjx_sim_destroy(mjxSim* sim);

/* One mj_step (forward + implicitfast/Euler integration) for every world, repeated
 * `nsubstep` times (ctrl/xfrc/qfrc_applied held fixed).  The state (qpos, qvel, act, time,
 * qacc_warmstart) advances every substep; the derived mjData outputs -- frames, contacts,
 * forces, subtree momenta and sensordata -- are the last substep's, computed in that substep
 * only (the contact sensors run every substep: the contact air times read their counts). */
int mjx_step(mjxSim* sim, int nsubstep, void* stream);
/* mj_forward without integration (kinematics/sensors/acc for the current state). */
int mjx_forward(mjxSim* sim, void* stream);
/* mj_forward only on worlds where mask[w] != 0 (mask: device uint8[nworld]; NULL = all).
 * Lets a sync-free (graph-captured) env step refresh just the worlds it reset. */
int mjx_forward_masked(mjxSim* sim, const uint8_t* mask, void* stream);
/* mj_resetData on worlds where mask[w] != 0 (mask: device uint8[nworld]; NULL = all). */
int mjx_reset(mjxSim* sim, const uint8_t* mask, void* stream);

/* Field access.  Data fields have a leading nworld dimension; model fields a
 * leading dimension of 1 (shared, world stride 0) or nworld after expansion.
 * The returned DLManagedTensor aliases library memory (float32/int32 on the sim's
 * device); call its deleter when done.  Pointers are stable for the sim's
 * lifetime except that mjx_expand_field reallocates that model field. */
struct DLManagedTensor;
int mjx_field(mjxSim* sim, const char* name, struct DLManagedTensor** out);
int mjx_field_count(const mjxSim* sim);
const char* mjx_field_name(const mjxSim* sim, int i);
int mjx_expand_field(mjxSim* sim, const char* name, void* stream);
int mjx_field_is_expanded(const mjxSim* sim, const char* name);

/* Contact-sensor air-time tracking inside the step (ContactSensor._update_air_time_tracking,
 * sensor/contact_sensor.py:327-367): after every integrated substep, for each of the `n`
 * tracked slots (n <= 8) with its `found` value at sensordata[found_adr[i]], update the
 * device buffers cur_air / last_air / cur_contact / last_contact [nworld, n] with the
 * elapsed time = time - last_time[w], then last_time[w] = time.  mjx_forward does not
 * update them.  found_adr is a host array; n = 0 turns tracking off.  Synchronises. */
int mjx_sim_track_air_time(mjxSim* sim, int n, const int32_t* found_adr, float* cur_air,
                           float* last_air, float* cur_contact, float* last_contact,
                           float* last_time, void* stream);

/* Diagnostics: per-sim counters as int32[8] written to host `out` ([0] max contacts, [1] max
 * rows seen, [2] contact-overflow, [3] row-overflow, [4] unsupported-pair events -- dropped
 * work --, [5] max Newton iterations, [6] worlds re-solved at the max capacity); synchronises
 * the stream. */
int mjx_sim_stats(mjxSim* sim, int32_t* out, void* stream);
/* The sim's capacities and kernels as int32[8]: [0] nconmax, [1] njmax (the fast carve),
 * [2] nconmax_max, [3] njmax_max, [4] spec of the fast carve's kernels, [5] spec of the max
 * capacity's kernels (csrc/specs.inc entry, 0 = generic), [6] re-solve list capacity per
 * substep, [7] Newton row classes. */
int mjx_sim_info(const mjxSim* sim, int32_t* out);
/* Diagnostics (parity tests): the joint-space inertia M of every world as the last substep's
 * phase A formed it (mjData.qM, mj_crb + armature; the reference reads it from mujoco_warp's
 * Data.qM), copied from the engine's phase hand-off scratch into the device buffer `out`:
 * float [nworld][L] with L = 8 nb (nb + 1), nb = ceil(nv / 4), the lower 4 x 4 tiles of the
 * nvp x nvp matrix row by row (row i = 4b + r holds columns [0, 4(b + 1)) at 8 b (b + 1) +
 * 4 (b + 1) r).  `big` = 1 reads the max-capacity scratch (worlds the overflow re-solve ran).
 * Valid after mjx_step / mjx_forward until the next launch; stream-ordered. */
int mjx_sim_mass_matrix(mjxSim* sim, int big, float* out, void* stream);
/* Diagnostics: per-stage cycle sums uint64[48] (non-zero only in the -DMJX_STAMPS build). */
int mjx_sim_profile(mjxSim* sim, uint64_t* out, void* stream);
/* Which step kernels the sim launches: k > 0 = kernels compiled for entry k of
 * csrc/specs.inc (the sim's dims, nconmax and njmax equal that entry), 0 = the generic
 * kernels; -1 for a null sim.  No reference counterpart (mujoco_warp specialises by
 * tracing Python at graph-capture time, sim/sim.py:164-191). */
int mjx_sim_spec(const mjxSim* sim);
/* Load a run-time specialisation: `path` is a shared library built from csrc/jit.hip for one
 * model's dims (mjlab_amd/jit.py compiles it with hipcc when a Simulation's model matches no
 * compiled csrc/specs.inc entry, and caches it).  Returns the specialisation id (>= 1000; a sim
 * created afterwards with those dims runs its kernels, mjx_sim_spec) or -1.  No reference
 * counterpart: mujoco_warp specialises kernels for any model by tracing at graph-capture
 * time (sim/sim.py:164-191); this is the AOT-compiled equivalent.  A library built from other
 * kernel headers than this engine (its mjx_jit_hdr differs from csrc/Makefile's MJX_HDR_HASH)
 * is refused (-1): its kernels would read the launch parameters through another layout. */
int mjx_spec_register(const char* path);
/* Diagnostics: enqueue one empty kernel (`mjx::marker_kernel`, one wave, argument `tag`) on
 * `stream`.  bench.py brackets its timed region with tags 1 and 2 outside the timing, so a
 * rocprofv3 kernel trace or --pmc pass of the same command can attribute exactly the
 * timed steps' dispatches.  No reference counterpart. */
int mjx_marker(int tag, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MJX355_H_ */
