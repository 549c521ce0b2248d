// fields.h — single source of truth for the device model/data field tables.
//
// X(name, count, width): `count` is an expression over the model dims struct `d`
// (mjxDims) and `width` the per-element width.  The same lists generate the device
// structs (engine.hip), the upload code and the DLPack field table (capi.cpp), so the
// Python-visible names match mjModel / mjData (sim/sim_data.py:177-240 exposes the
// same names from MuJoCo-Warp).
#pragma once

// Model integer fields (never expanded per world).
#define MJX_MODEL_INT_FIELDS(X)                                                        \
  X(body_parentid, d.nbody, 1) X(body_rootid, d.nbody, 1) X(body_weldid, d.nbody, 1) \
  X(body_jntnum, d.nbody, 1) X(body_jntadr, d.nbody, 1) X(body_dofnum, d.nbody, 1)   \
  X(body_dofadr, d.nbody, 1) X(body_level, d.nbody, 1)                               \
  X(body_childadr, d.nbody + 1, 1) X(body_child, d.nchild, 1)                         \
  X(body_mocapid, d.nbody, 1) X(level_start, d.nlevel + 1, 1) X(level_body, d.nbody, 1) \
  X(jnt_type, d.njnt, 1) X(jnt_qposadr, d.njnt, 1) X(jnt_dofadr, d.njnt, 1)          \
  X(jnt_bodyid, d.njnt, 1) X(jnt_limited, d.njnt, 1)                                 \
  X(dof_bodyid, d.nv, 1) X(dof_jntid, d.nv, 1) X(dof_parentid, d.nv, 1)              \
  X(geom_type, d.ngeom, 1) X(geom_bodyid, d.ngeom, 1) X(geom_contype, d.ngeom, 1)    \
  X(geom_conaffinity, d.ngeom, 1) X(geom_condim, d.ngeom, 1)                         \
  X(geom_priority, d.ngeom, 1) X(geom_dataid, d.ngeom, 1)                            \
  X(site_bodyid, d.nsite, 1) X(actuator_trnid, d.nu, 1)                              \
  X(actuator_forcelimited, d.nu, 1) X(actuator_ctrllimited, d.nu, 1)                 \
  X(sensor_type, d.nsensor, 1) X(sensor_objtype, d.nsensor, 1)                       \
  X(sensor_objid, d.nsensor, 1) X(sensor_reftype, d.nsensor, 1)                      \
  X(sensor_refid, d.nsensor, 1) X(sensor_adr, d.nsensor, 1) X(sensor_dim, d.nsensor, 1) \
  X(sensor_intprm, d.nsensor, 3) X(pair_geom1, d.npair, 1) X(pair_geom2, d.npair, 1) \
  X(hfield_nrow, d.nhfield, 1) X(hfield_ncol, d.nhfield, 1) X(hfield_adr, d.nhfield, 1)

// Model float fields: uploaded as fp32, each may be expanded to one copy per world
// (Simulation.expand_model_fields, sim/sim.py:226-240).
#define MJX_MODEL_FLOAT_FIELDS(X)                                                      \
  X(body_pos, d.nbody, 3) X(body_quat, d.nbody, 4) X(body_ipos, d.nbody, 3)          \
  X(body_iquat, d.nbody, 4) X(body_mass, d.nbody, 1) X(body_inertia, d.nbody, 3)     \
  X(body_subtreemass, d.nbody, 1) X(body_invweight0, d.nbody, 2)                     \
  X(jnt_pos, d.njnt, 3) X(jnt_axis, d.njnt, 3) X(jnt_range, d.njnt, 2)               \
  X(jnt_solref, d.njnt, 2) X(jnt_solimp, d.njnt, 5) X(jnt_margin, d.njnt, 1)         \
  X(jnt_stiffness, d.njnt, 1) X(qpos0, d.nq, 1) X(qpos_spring, d.nq, 1)              \
  X(dof_armature, d.nv, 1) X(dof_damping, d.nv, 1) X(dof_invweight0, d.nv, 1)        \
  X(dof_frictionloss, d.nv, 1)                                                       \
  X(geom_size, d.ngeom, 3) X(geom_pos, d.ngeom, 3) X(geom_quat, d.ngeom, 4)          \
  X(geom_friction, d.ngeom, 3) X(geom_solmix, d.ngeom, 1) X(geom_solref, d.ngeom, 2) \
  X(geom_solimp, d.ngeom, 5) X(geom_margin, d.ngeom, 1) X(geom_gap, d.ngeom, 1)      \
  X(geom_rbound, d.ngeom, 1) X(site_pos, d.nsite, 3) X(site_quat, d.nsite, 4)        \
  X(actuator_gear, d.nu, 1) X(actuator_gainprm, d.nu, 3) X(actuator_biasprm, d.nu, 3) \
  X(actuator_forcerange, d.nu, 2) X(actuator_ctrlrange, d.nu, 2)                     \
  X(hfield_size, d.nhfield, 4) X(hfield_data, d.nhfielddata, 1)

// Per-world data fields, fp32, layout [nworld][count*width] (torch row-major).
#define MJX_DATA_FLOAT_FIELDS(X)                                                       \
  X(qpos, d.nq, 1) X(qvel, d.nv, 1) X(qacc, d.nv, 1) X(qacc_warmstart, d.nv, 1)       \
  X(qacc_smooth, d.nv, 1) X(ctrl, d.nu, 1) X(time, 1, 1) X(qfrc_applied, d.nv, 1)    \
  X(xfrc_applied, d.nbody, 6) X(mocap_pos, d.nmocap, 3) X(mocap_quat, d.nmocap, 4)    \
  X(xpos, d.nbody, 3) X(xquat, d.nbody, 4) X(xmat, d.nbody, 9) X(xipos, d.nbody, 3)  \
  X(ximat, d.nbody, 9) X(cvel, d.nbody, 6) X(cacc, d.nbody, 6)                       \
  X(subtree_com, d.nbody, 3) X(subtree_linvel, d.nbody, 3)                            \
  X(subtree_angmom, d.nbody, 3) X(geom_xpos, d.ngeom, 3) X(geom_xmat, d.ngeom, 9)    \
  X(site_xpos, d.nsite, 3) X(site_xmat, d.nsite, 9) X(sensordata, d.nsensordata, 1)  \
  X(actuator_force, d.nu, 1) X(actuator_length, d.nu, 1) X(actuator_velocity, d.nu, 1) \
  X(qfrc_actuator, d.nv, 1) X(qfrc_bias, d.nv, 1) X(qfrc_passive, d.nv, 1)            \
  X(qfrc_constraint, d.nv, 1) X(qfrc_smooth, d.nv, 1)                                \
  X(contact_dist, d.nconmax, 1) X(contact_pos, d.nconmax, 3) X(contact_frame, d.nconmax, 9)   \
  X(contact_force, d.nconmax, 3)

#define MJX_DATA_INT_FIELDS(X) \
  X(ncon, 1, 1) X(nefc, 1, 1) X(solver_niter, 1, 1) X(contact_geom, d.nconmax, 2)
