// engine.h — device-side model/data descriptors and kernel launchers of the mjx355
// HIP engine (gfx950).  Host code (capi.cpp) fills these structs; engine.hip reads
// them.  Layout and ownership are described in DESIGN.md section 3.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fields.h"

namespace mjx {

constexpr int kWave = 64;        // CDNA wavefront width
// contacts per world: a fast carve holds at most one per lane (<= kWave); a max (re-solve)
// carve up to kMaxContacts, kMaxConRounds per lane
constexpr int kMaxConRounds = 8;
constexpr int kMaxContacts = kWave * kMaxConRounds;
constexpr int kBodyRec = 20, kDofRec = 12, kActRec = 4;  // ints per DModel record (int4-aligned)
constexpr int kMaxBodies = 64;   // dof_bodymask is uint64
constexpr int kMaxDof = 64;      // one lane per dof in the dof-parallel stages
constexpr int kMaxLanes = 64;    // nu, njnt: one lane per actuator / joint (register records)
constexpr int kRowClasses = 2;   // Newton row classes below the full capacity
constexpr int kMaxSplit = 4;     // concurrent batch splits (launch_step; default 2)
constexpr int kSplitMinWorlds = 2048;  // batches at least this large run split
constexpr int kMaxAirSlots = 8;  // contact-sensor slots with air-time tracking
constexpr int kStaticChunk = 64; // terrain geoms per broadphase chunk

enum { EFC_LIMIT = 0, EFC_FRICTIONLESS = 1, EFC_PYRAMIDAL = 2 };
enum { GEOM_PLANE = 0, GEOM_HFIELD = 1, GEOM_SPHERE = 2, GEOM_CAPSULE = 3, GEOM_BOX = 6 };
enum { JNT_FREE = 0, JNT_BALL = 1, JNT_SLIDE = 2, JNT_HINGE = 3 };
enum { SENS_GYRO = 0, SENS_VELOCIMETER = 1, SENS_ACCELEROMETER = 2, SENS_SUBTREEANGMOM = 3,
       SENS_CONTACT = 4, SENS_FRAMEPOS = 5, SENS_FRAMEQUAT = 6, SENS_JOINTPOS = 7,
       SENS_JOINTVEL = 8 };
enum { OBJ_SITE = 6 };
enum { REDUCE_NONE = 0, REDUCE_MINDIST = 1, REDUCE_MAXFORCE = 2, REDUCE_NETFORCE = 3 };

struct Dims {
  int nq, nv, nu, nbody, njnt, ngeom, nsite, nsensor, nsensordata, npair;
  int nhfield, nhfielddata, nlevel, nchild, nmocap;
  int ngeom_lds;  // geoms whose world frames phase A keeps in LDS (all but static terrain geoms)
  int npair_all;  // pair list length: [0, npair) regular pairs, [npair, npair_all) terrain pairs
  int nstatic;    // static terrain geoms (heightfields, world-welded boxes) with candidate pairs
  int nstpartner; // distinct geoms paired with a terrain geom (their union AABB culls terrain)
  int nboxbox;    // box-box candidate pairs: kernels specialised for a model without any are
                  // compiled without the box-box narrowphase (its registers cost occupancy)
  int nconmax;  // contacts per world held in LDS
  int njmax;    // constraint rows per world held in LDS
};

struct Opt {
  float timestep, tolerance, ls_tolerance, impratio, meaninertia;
  float gravity[3];
  int iterations, ls_iterations, integrator, cone;
  int maxmatch;  // contact-sensor matches per sensor and world (the first ones in contact order)
};

// Device model: int fields shared, float fields with a per-world stride (0 = shared).
struct DModel {
#define X_INT(name, cnt, w) const int32_t* name;
#define X_FLT(name, cnt, w) const float* name; int name##_ws;
  MJX_MODEL_INT_FIELDS(X_INT)
  MJX_MODEL_FLOAT_FIELDS(X_FLT)
#undef X_INT
#undef X_FLT
  const uint64_t* dof_bodymask;
  const uint64_t* dof_ancmask;  // bit j set: dof j is dof i itself or an ancestor (host-derived)
  const uint64_t* body_submask;  // bit c set: body c is in body b's subtree (b included)
  const uint64_t* body_dofmask;  // bit j set: dof j moves body b (dofs of b and its ancestors)
  // per-lane model records, host-packed (capi.cpp, kBodyRec / kDofRec / kActRec ints each):
  // the integer part of load_body / the dof record / load_act in one contiguous record, so
  // a lane's float loads depend on ONE load instead of a chain (level_body -> body_* ->
  // jnt_* -> qpos0).  body_rec is in level order (record i = level-order body i).
  const int32_t* body_rec;
  const int32_t* dof_rec;
  const int32_t* act_rec;
  // host-derived terrain broadphase tables (capi.cpp).  Static terrain geoms (heightfields,
  // boxes welded to the world) keep no LDS frame: geom_lds = -1, lds_geom its inverse over
  // the others.  st_geom lists the terrain geoms with pairs, in pair-tail order; their pair
  // blocks are [st_pairadr[i], st_pairadr[i+1]); st_aabb holds each one's world AABB (lo xyz,
  // hi xyz, margin included) and st_chunk_aabb the union over chunks of kStaticChunk
  // consecutive ones; st_partner lists the distinct partner geoms.
  const int32_t* geom_lds;
  const int32_t* lds_geom;
  const int32_t* st_geom;
  const int32_t* st_pairadr;
  const int32_t* st_partner;
  const float* st_aabb;
  const float* st_chunk_aabb;
  // regular pairs as one 16-B record each (capi.cpp): {g1 | g2 << 16, l1 | l2 << 12 |
  // t1 << 24 | t2 << 28 (LDS frame slots, geom types), margin, bounding-sphere cull radius
  // r1 + r2 + margin (+inf: no cull)}; null when ids exceed the packing.  Valid while
  // geom_rbound / geom_margin are not expanded per world.
  const int32_t* pair_rec;
  int nmaskword;  // 32-bit words per contact-sensor geom mask
  const uint32_t* sensor_geommask1;
  const uint32_t* sensor_geommask2;
  // single-slot contact sensors, transposed (host-derived): geom_csmask{1,2}[g] bit k is set
  // when geom g is in the primary / secondary set of the k-th such sensor (cs_sensor[k]); a
  // contact then finds every sensor it matches from two 64-bit loads per geom
  int ncsens;
  const int32_t* cs_sensor;
  const uint64_t* geom_csmask1;
  const uint64_t* geom_csmask2;
};

struct DData {
#define X_FLT(name, cnt, w) float* name;
#define X_INT(name, cnt, w) int32_t* name;
  MJX_DATA_FLOAT_FIELDS(X_FLT)
  MJX_DATA_INT_FIELDS(X_INT)
#undef X_FLT
#undef X_INT
  int32_t* stats;   // [8] reduced engine counters (filled by mjx_sim_stats)
  int32_t* wstats;  // [nworld][8] per-world counters (no cross-world atomics in the kernels)
  int32_t* evtotal; // [4] overflow / unsupported-pair events over all worlds (an atomic per
                    // event, and events are rare: no per-substep cross-world traffic)
  unsigned long long* prof;  // [48] stage cycle sums (diagnostic -DMJX_STAMPS build)
  unsigned long long* wtrace;  // [nworld][8] per-world phase start/end s_memrealtime (MJX_STAMPS)
};

// Per-world LDS carve (offsets in 4-byte words).
struct Lds {
  int qpos, qvel, ctrl, qacc_ws, qfrc_applied, xfrc;
  int xpos, xquat, xmat, xipos, ximat, xanchor, xaxis;
  int stmass, subtree_com, cinert, crb, cvel, cacc, stlin, stang;
  int cdof, cdofdot, cacc_v, gxpos, gxmat, sxpos, sxmat;
  int M, H;
  int qfrc_bias, qfrc_passive, qfrc_act, qfrc_smooth, qacc_smooth, x, Mx, grad, srch, Ms,
      qfrc_con, vtmp, act_force, act_len, act_vel;
  int con_g1, con_g2, con_key, con_dist, con_pos, con_frame, con_mu, con_kb,
      con_imp, con_imargin, con_dim, con_efc, con_n;
  int efc_J, efc_aref, efc_D, efc_jar, efc_Js, efc_force, efc_cid, efc_act, hdiag;
  int red;      // 5*kWave scratch (J^T w partial sums)
  int chol;     // 4*NR floats: column blocks of the blocked Cholesky (rows_chol)
  int ints;     // small int block: [0]=raw ncon [1]=nefc [2]=nlimit [3]=flags [4]=ncon [5]=niter
  int pack_len; // length of the phase's input pack (carved first; see make_lds)
  int packC_b;  // C carve: offset of the part of the pack written by phase B
  int packC_sub; // C carve: end of the part every substep reads (the rest: the last substep's)
  int total;
};

}  // namespace mjx
#include "carve.h"  // constexpr Lds make_lds(const Dims& d, int phase): phase 0/1/2 = A/B/C
namespace mjx {

// Model specialisation: 0 = generic kernels (dims and carves read from Params at run
// time), k > 0 = kernels compiled for the k-th entry of specs.inc (dims and carves are
// compile-time constants).  find_spec returns the entry equal to d in every field and in
// the dof tree (dof_parentid, for the tree-form SPD factors), else 0.
constexpr int kMaxSpecs = 8;
int find_spec(const Dims& d, const int* dof_parentid);
// Specialisations compiled at run time (jit.hip, loaded by mjx_spec_register) get ids from
// kRtSpecBase on; find_spec checks them after the compiled specs.inc entries.
constexpr int kRtSpecBase = 1000;
using StepFnPtr = void (*)(const struct Params*, int, int, int, int, int, const uint8_t*);
int register_spec(const Dims& d, const int* par, int npar, StepFnPtr (*fn)(int));

// Everything a launch needs, resident in device memory (read through the scalar cache
// instead of occupying ~500 SGPRs of kernarg space).
struct Params {
  Dims d;
  Opt o;
  DModel m;
  DData D;
  // Per-phase LDS carves: [0] A, [1] B at full row capacity, [2] C, [3 + k] B for Newton row
  // class k.  Worlds whose nefc fits class k's capacity run Newton in its smaller carve (more
  // resident worlds per CU); classes run concurrently (launch_step).
  Lds LP[3 + kRowClasses];
  Lds LPJ;  // phase B at full capacity with J read from the B pack in global memory (kLdsJG)
  int nrowclass;                 // row classes in use (0 = every world in LP[1])
  int row_cap[kRowClasses];      // ascending row capacities of the classes
  // Newton work lists (classify_kernel, every substep between phases A and B): worlds sorted
  // by constraint-row count, descending; row class k's worlds are wl_list[wl_seg[2k] ..
  // wl_seg[2k] + wl_seg[2k+1]) -- each class launch takes its worlds densely and largest
  // first instead of filtering all nworld workgroups.
  int* wl_list;
  int* wl_seg;   // [kMaxSplit][2 * (kRowClasses + 1)]: one segment table per batch split
  float* gscr;   // per-world hand-off scratch: [B pack | C pack | F], gstride floats per world
  int gC;        // offset of the C pack inside a world's scratch
  int gF;        // offset of F: the implicit-integration factor (nvp x nvp rows), read by
                 // phase C straight from global memory (not staged in LDS)
  int gstride;
  int spec;      // model specialisation (find_spec) whose kernels launch_step uses
  // contact-sensor air-time tracking (mjx_sim_track_air_time): phase C of every integrated
  // substep updates nair slots per world from sensordata[air_found[i]]
  int nair;
  int air_found[kMaxAirSlots];
  float *air_cur, *air_last, *air_cc, *air_lc, *air_time;
  int stamp_minrows;  // diagnostic stamps build: count worlds with at least this many rows
  // Overflow re-solve ("Contact budget"): with ovf_resolve set, a world
  // whose contacts or constraint rows overflow this carve is not truncated -- phase A lists
  // it (ovf_list / ovf_n, one list per batch split and substep parity, ovf_cap entries each)
  // and flags it (ovf_flag[w], rewritten by the world's every phase A), skips the rest of
  // its substep in this carve, and the "max" launch set (a second Params at the sim's full
  // capacity) re-solves its substep from its state.  The max Params have ovf_resolve = 0:
  // what overflows them is dropped and counted.
  int ovf_resolve;
  int outputs_every;  // diagnostic (MJX355_OUTPUTS_EVERY=1): sensors / subtree momenta every substep
  int ovf_cap;
  int* ovf_list;   // [kMaxSplit][2][ovf_cap]
  int* ovf_n;      // [kMaxSplit][2]
  int* ovf_flag;   // [nworld]
  int* ovf_done;   // [kMaxSplit][2] workgroups through the list's last launch (it clears the list)
  int con_stride;  // contact slots per world of the contact output arrays (the max capacity)
};

// `sel` launch argument of the step kernels: bits 0-7 batch split, 8-15 row class + 1 (the
// piped C / next-A launches of a class), kSelOvf: the world is the blockIdx-th entry of the
// overflow list of parity kSelRPar, kSelAPar: the parity of the substep phase A computes
// (the list it appends overflowing worlds to).
// workgroups of a re-solve launch (each loops over listed worlds).  Measured (G1 4,096 at a
// 20-contact / 80-row fast carve, 3.5 % of world-substeps re-solved): 64 workgroups 1.43 M
// env-steps/s, 256 1.69 M, 512 1.65 M; with nothing listed the grid size is not measurable.
constexpr int kOvfGrid = 256;
// ... and where the chain runs in line behind a range chain or on a split stream (the critical
// path).  There the launch dispatches while the other range's chain holds every CU (Go1 16 / 64:
// 16 worlds per CU, the register file full at 4 waves per SIMD), and each max-carve workgroup
// (32 KB of LDS, 256 VGPRs) waits for several of that chain's waves to retire: the empty launch
// spans 20-34 us (kernel trace, profiles/r06_go1_step_timeline.txt).  Go1 flat 8,192, two
// interleaved rounds: 32 workgroups 8.71 / 8.68 M env-steps/s, 1 workgroup 8.93 / 8.88 M, no
// re-solve at all (MJX355_RESOLVE=0, the bound) 9.24 / 9.13 M; round 4 (24 / 96 carve): 256 /
// 64 / 32 / 16 workgroups 6.73 / 7.32 / 7.40 / 7.41 M.  The price: the one workgroup re-solves
// the listed worlds one after another (forced overflow, G1 split at a 20 / 80 carve, round 4:
// 64 / 32 / 16 workgroups 1.49 / 1.17 / 0.81 M), so a range-chained batch whose fast carve
// overflows often should get a larger carve (Simulation.fast_capacity, the bench's
// overflow.resolved_events); MJX355_OVF_GRID overrides.
constexpr int kOvfGridInline = 1;
constexpr int kSelOvf = 1 << 16;
constexpr int kSelAPar = 1 << 17;
constexpr int kSelRPar = 1 << 18;
constexpr int kSelClr = 1 << 19;  // the re-solve launch that empties its list on exit
// the fused class-chain launch (step_chain: one world's Newton, phase C and the next
// substep's phase A back to back): kSelChainA runs that phase A, kSelNextLast marks the
// next substep as the step's last; kSelFusedA: a phase A that follows phase C in the same
// launch (it reads the state C just stored past the vector L1)
constexpr int kSelChainA = 1 << 20;
constexpr int kSelNextLast = 1 << 21;
constexpr int kSelFusedA = 1 << 22;
// the full-capacity class's launches (engine.hip heavy_cap): its waves raise their issue
// priority (s_setprio) over the bulk-class waves sharing their SIMDs
constexpr int kSelPrio = 1 << 23;

// Launchers (enqueue on `stream`; never synchronise).  `dev` points to a device copy of
// `host`; `host` is used only for the launch geometry.
hipError_t prepare_step(const Params& host);  // one-time kernel attributes (not capturable)
// Side streams for the Newton row classes beyond the first: forked from and joined back
// into the split's stream every substep (graph-capturable fork/join).
// With the batch split (nsplit > 1), split k > 0 runs on split[k], forked from the launch
// stream before the first substep and joined back after the last.  Every split owns its
// class streams and fork / join events, so the captured dependency graph is a tree of
// per-split fork/join diamonds (class streams shared by two splits made a capture whose
// side streams joined two origin streams, and hipStreamEndCapture crashed on it).
struct SideStream {
  hipStream_t stream[kMaxSplit][kRowClasses];
  hipEvent_t fork[kMaxSplit], join[kMaxSplit][kRowClasses];
  int nsplit;                        // batch splits in use (1 = one launch set per phase)
  hipStream_t split[kMaxSplit];      // [0] unused: split 0 runs on the launch stream
  hipEvent_t split_fork, split_join[kMaxSplit];
  // overflow re-solve chain of each split (forked after phase A / classify, joined before the
  // next substep's classify)
  hipStream_t ovf[kMaxSplit];
  hipEvent_t ovf_fork[kMaxSplit], ovf_join[kMaxSplit];
  bool range_chain = false;  // models without row classes: range_chain_default
};
// Whether a model without row classes runs each batch range's B -> C -> next A as one
// launch (engine.hip launch_step; MJX355_RANGE_CHAIN=0/1 overrides).
bool range_chain_default(const struct Params& host, int nworld, int nsplit);
// `hbig` / `dbig`: the max-capacity Params (host copy for the launch geometry, device copy
// for the kernels) of the overflow re-solve, or null (overflow drops contacts).
hipError_t launch_step(const Params& host, const Params* dev, int nworld, int nsubstep,
                       int integrate, const uint8_t* mask, hipStream_t stream,
                       const SideStream* side, const Params* hbig = nullptr,
                       const Params* dbig = nullptr);
// Newton row classes (capacities ascending into caps[]); returns how many are used.
int choose_row_classes(const Dims& d, int spec, int (&caps)[kRowClasses]);
hipError_t launch_reset(const Dims& d, const DModel& m, const DData& dd, const uint8_t* mask,
                        int nworld, int con_stride, hipStream_t stream);
hipError_t launch_marker(int tag, hipStream_t stream);  // empty kernel (profiling brackets)

}  // namespace mjx
