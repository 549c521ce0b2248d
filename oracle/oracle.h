/* oracle.h — CPU (fp64) restatement of the mj_step pipeline subset on the hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the reported CPU
 * baseline.  The product path (mjlab-1_amd) never links or calls it.
 *
 * Parity status: the reference's physics lives in un-vendored mujoco_warp (git
 * f2f7957) / MuJoCo 3.4.1.dev and neither is importable here,
 * so this restatement is pinned by (a) the reference's own known-answer tests
 * (tests/test_spec_utils.py:26-102 actuator law, tests/test_sim.py:89-110 reset,
 * tests/test_entity_data.py:44-158 velocity round trips) re-expressed in tests/,
 * and (b) analytic answers (free fall, pendulum, box-on-plane m*g).  Trajectory
 * parity with MuJoCo-C itself is UNPINNED (no MuJoCo in the container).
 */
#ifndef MJX_ORACLE_H_
#define MJX_ORACLE_H_

#include "../include/mjx355.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int geom1, geom2, dim;
  double dist, includemargin;
  double pos[3], frame[9];
  double friction[5], solref[2], solimp[5];
  int efc_address;
} orcContact;

typedef struct {
  int nconmax, njmax;
  /* state (in) */
  double time;
  double *qpos, *qvel, *qacc_warmstart, *ctrl, *qfrc_applied, *xfrc_applied;
  /* position stage */
  double *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis;
  double *geom_xpos, *geom_xmat, *site_xpos, *site_xmat;
  double *subtree_com, *cinert, *cdof, *crb, *qM;
  /* velocity stage */
  double *cvel, *cdof_dot, *qfrc_bias, *qfrc_passive, *subtree_linvel, *subtree_angmom;
  /* actuation / acceleration */
  double *actuator_force, *qfrc_actuator, *qfrc_smooth, *qacc_smooth;
  double *qacc, *qfrc_constraint, *cacc, *sensordata;
  /* contacts + constraints */
  int ncon, nefc, niter, nlimit;
  orcContact* contact;
  int *efc_type, *efc_id;
  double *efc_J, *efc_pos, *efc_margin, *efc_D, *efc_R, *efc_aref, *efc_vel, *efc_force,
      *efc_diagApprox, *efc_frame_mu;
  int overflow; /* bit0: contacts dropped, bit1: rows dropped, bit2: unsupported pair */
  /* when set: the constraint stage takes qacc from here instead of running the Newton
   * solver (forces, qfrc_constraint and the integration follow from it) */
  const double* qacc_given;
  const double* qfrc_constraint_given;  /* with qacc_given: the integration uses this */
  const double* qfrc_smooth_given;      /* with qacc_given: and this */
  const double* qM_given;               /* with qacc_given (may be NULL): the integration's M */
  double cost;  /* the constraint-problem cost at the final qacc (Gauss + active rows) */
  /* scratch */
  double* work;
} orcData;

orcData* orc_data_new(const mjxModelDesc* m, int nconmax, int njmax);
void orc_data_free(orcData* d);
void orc_reset(const mjxModelDesc* m, orcData* d);      /* mj_resetData */
void orc_forward(const mjxModelDesc* m, orcData* d);    /* mj_forward */
void orc_step(const mjxModelDesc* m, orcData* d);       /* mj_step (implicitfast/euler) */

/* Batched helpers for the Python tests / CPU baseline: worlds are independent; the
 * state arrays are [nworld][n] contiguous.  Runs `nstep` steps per world, copying the
 * selected outputs back.  nthreads<=0: all cores (OpenMP). */
int orc_rollout(const mjxModelDesc* m, int nworld, int nstep, int nconmax, int njmax,
                double* qpos, double* qvel, double* qacc_warmstart, double* ctrl,
                double* time, double* qacc_out, double* sensordata_out,
                double* xpos_out, double* cvel_out, double* subtree_com_out,
                double* actuator_force_out, int* ncon_out, int nthreads);

/* Single-world full data dump for parity tests (all pointers may be NULL). */
int orc_forward_dump(const mjxModelDesc* m, int nconmax, int njmax, const double* qpos,
                     const double* qvel, const double* qacc_warmstart, const double* ctrl,
                     double time, int do_step, double* out_qpos, double* out_qvel,
                     double* out_qacc, double* out_qacc_smooth, double* out_sensordata,
                     double* out_xpos, double* out_xquat, double* out_cvel,
                     double* out_subtree_com, double* out_qfrc_bias, double* out_qM,
                     double* out_actuator_force, double* out_cacc, int* out_ncon,
                     int* out_nefc, double* out_contact /* ncon*(2+1+3+3) */,
                     double* out_efc_force, int* out_niter);

/* One mj_step whose constraint stage uses the given qacc instead of solving for it:
 * efc_force = -D (J qacc - aref) on the rows with J qacc < aref, qfrc_constraint = J^T f,
 * then the implicitfast / Euler integration of orc_step.  The parity tests use it to check
 * the engine's integration against its own solver output (the solver is checked
 * separately through qacc). */
int orc_step_given_qacc(const mjxModelDesc* m, int nconmax, int njmax, const double* qpos,
                        const double* qvel, const double* qacc_warmstart, const double* ctrl,
                        double time, const double* qacc, const double* qfrc_constraint,
                        const double* qfrc_smooth, const double* qM, double* out_qpos,
                        double* out_qvel, double* out_sensordata, double* out_qfrc_constraint,
                        double* out_cost, double* out_efc_force /* njmax */, int* out_nefc);

/* fp32 error scale of the Newton solution: mj_forward (fp64 solve), then at the solution
 * x the Hessian H = M + J_a^T D_a J_a of the active rows and, per dof j, the magnitude of
 * the gradient's terms a_j = sum_r |J_rj D_r jar_r| + sum_k |M_jk x_k| + |qfrc_smooth_j|
 * (what an fp32 gradient evaluation rounds); out_scale[i] = sum_j |H^-1_ij| a_j.  A solver
 * whose gradient is exact to eps relative to its terms lands within eps * out_scale of x.
 * out_vscale (may be NULL): the same for the implicit integration's velocity update,
 * h * sum_j |A^-1_ij| (|qfrc_smooth_j| + |qfrc_constraint_j| + sum_k |A_jk dv_k|) with
 * A = M + h D (the implicitfast matrix) and dv the update.  a_extra (may be NULL) is added
 * to a_j: a perturbation of the problem data already divided by eps (the parity tests pass
 * the engine's measured mass-matrix and smooth-force differences, |dM| |x| + |d qfrc_smooth|,
 * so the scale covers a solver that solved the engine's problem exactly to rounding). */
int orc_qacc_error_scale(const mjxModelDesc* m, int nconmax, int njmax, const double* qpos,
                         const double* qvel, const double* qacc_warmstart, const double* ctrl,
                         double time, const double* a_extra, double* out_scale,
                         double* out_vscale);

/* Magnitude of the terms an evaluation of M sums (the composite-rigid-body algorithm about
 * the root's subtree com, MuJoCo's mj_crb / cinert / cdof convention, as the engine forms
 * it): out_Mabs[i][j] = |cdof_j| . (|crb_abs(body(i))| |cdof_i|), with crb_abs the subtree
 * sum of each body's cinert term magnitudes (|I_c| + m (|d|^2 + d_k^2), m |d_k d_l|, m |d_k|,
 * m) and every product taken in absolute value; armature on the diagonal.  A finite-
 * precision M is exact to (a few) eps times this, not times |M|: a light dof deep in a tree
 * (an ankle roll) is a small difference of O(m d^2) terms. */
int orc_mass_matrix_scale(const mjxModelDesc* m, const double* qpos, double* out_Mabs);

/* fp32 evaluation scale of the Newton cost at the fp64 solution x (mj_forward first): the
 * magnitude of the terms eval_cost sums, 1/2 sum_i (|x_i| + |qacc_smooth_i|)(sum_k |M_ik x_k| +
 * |qfrc_smooth_i|) + sum_{active r} 1/2 D_r (sum_i |J_ri x_i| + |aref_r|)^2.  An fp32 solver
 * cannot tell costs apart closer than eps times this, so a cost gap between the engine's and
 * the oracle's qacc is judged in units of eps * out_scale -- not relative to the cost itself,
 * which is ~0 in a contact-free world (x = qacc_smooth minimises the Gauss term exactly). */
int orc_cost_scale(const mjxModelDesc* m, int nconmax, int njmax, const double* qpos,
                   const double* qvel, const double* qacc_warmstart, const double* ctrl, double time,
                   double* out_scale);

#ifdef __cplusplus
}
#endif
#endif
