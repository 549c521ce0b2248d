// capi.cpp — the extern "C" boundary declared in include/mjx355.h.
//
// Owns every device buffer (model blob, per-field data arrays, stats), hands out
// DLPack aliases, and enqueues the engine kernels on the caller's HIP stream.  The
// Python host mirror of mjlab.sim.Simulation (mjlab_amd/sim/sim.py) binds this with
// ctypes; INTEGRATION.md shows the same binding for other hosts.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <algorithm>
#include <vector>

#include "../../include/mjx355.h"
#include "engine.h"

// ---------------------------------------------------------------- minimal DLPack ABI
extern "C" {
typedef struct { int32_t device_type; int32_t device_id; } DLDevice;
typedef struct { uint8_t code; uint8_t bits; uint16_t lanes; } DLDataType;
typedef struct {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
} DLTensor;
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(struct DLManagedTensor*);
};
}
static const int32_t kDLROCM = 10;

namespace {
thread_local std::string g_err;
int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}
#define HIPCHK(expr)                                                                 \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) return fail(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct FieldInfo {
  void* ptr;
  bool is_float;
  int64_t count, width;
  bool per_world;     // data field (leading nworld) or expanded model field
  bool model;
  bool scalar = false;  // one value per world (time, ncon, ...): shape [nworld]
};
}  // namespace

struct mjxModel_ {
  int device;
  mjx::Dims d;
  mjx::Opt o;
  mjx::DModel dm;
  std::vector<void*> allocs;
  // host fp32 copies of float fields (defaults for expansion)
  std::map<std::string, std::vector<float>> host_float;
  std::vector<int> dof_parentid;  // host copy: find_spec checks a specialisation's dof tree
  std::map<std::string, std::pair<int64_t, int64_t>> float_dims;  // count, width
  std::map<std::string, std::pair<int64_t, int64_t>> int_dims;
  // static world frames of heightfield geoms (terrain bodies are welded to the world)
  std::vector<int> static_geoms;
  std::vector<float> static_xpos, static_xmat;
};

struct mjxSim_ {
  const mjxModel_* model;
  int nworld;
  mjx::Dims d;
  mjx::DModel dm;  // per-sim copy: expanded fields point to per-world buffers
  mjx::DData dd;
  mjx::Lds lds_ph[3 + mjx::kRowClasses];  // per-phase LDS carves ([3 + k]: Newton row class k)
  int nrowclass = 0;
  int row_cap[mjx::kRowClasses] = {};
  int nair = 0;  // contact air-time tracking (mjx_sim_track_air_time)
  int air_found[mjx::kMaxAirSlots] = {};
  float* air_buf[5] = {};
  int spec = 0;  // model specialisation in use (mjx::find_spec), 0 = generic kernels
  mjx::SideStream side{};  // streams of the Newton row classes (when classes are used)
  ~mjxSim_() {
    for (int p = 0; p < mjx::kMaxSplit; p++) {
      if (side.fork[p]) (void)hipEventDestroy(side.fork[p]);
      for (int k = 0; k < mjx::kRowClasses; k++) {
        if (side.join[p][k]) (void)hipEventDestroy(side.join[p][k]);
        if (side.stream[p][k]) (void)hipStreamDestroy(side.stream[p][k]);
      }
    }
    for (int p = 0; p < mjx::kMaxSplit; p++) {
      if (side.split[p]) (void)hipStreamDestroy(side.split[p]);
      if (side.split_join[p]) (void)hipEventDestroy(side.split_join[p]);
    }
    if (side.split_fork) (void)hipEventDestroy(side.split_fork);
    for (int p = 0; p < mjx::kMaxSplit; p++) {
      if (side.ovf[p]) (void)hipStreamDestroy(side.ovf[p]);
      if (side.ovf_fork[p]) (void)hipEventDestroy(side.ovf_fork[p]);
      if (side.ovf_join[p]) (void)hipEventDestroy(side.ovf_join[p]);
    }
  }
  int gC = 0, gF = 0, gstride = 0;
  float* gscr = nullptr;
  int* wl = nullptr;  // Newton work lists: [nworld] world ids + [kMaxSplit][2 * (kRowClasses + 1)] segments
  void* arena = nullptr;
  mjx::Params* dparams = nullptr;  // device copy of the launch parameters
  // overflow re-solve (mjx_sim_create_ex with a max capacity above the fast carve): the
  // max-capacity dims / carves / kernels / scratch, and the lists phase A fills
  bool big = false;
  mjx::Dims dbig{};
  mjx::Lds lds_big[3]{};
  int spec_big = 0;
  int gC_big = 0, gF_big = 0, gstride_big = 0;
  float* gscr_big = nullptr;
  int* ovf = nullptr;  // [kMaxSplit][2][ovf_cap] lists, [kMaxSplit][2] counts, [nworld] flags,
                       // [kMaxSplit][2] done counters
  int ovf_cap = 0;
  int con_stride = 0;  // contact slots per world in the contact output arrays
  mjx::Params* dparams_big = nullptr;
  std::vector<void*> expanded_allocs;
  std::map<std::string, FieldInfo> fields;
  std::vector<std::string> names;
  int32_t* stats = nullptr;
};

static mjx::Params host_params(const mjxSim_* s) {
  mjx::Params p;
  p.d = s->d;
  p.o = s->model->o;
  p.m = s->dm;
  p.D = s->dd;
  for (int i = 0; i < 3 + mjx::kRowClasses; i++) p.LP[i] = s->lds_ph[i];
  p.LPJ = mjx::make_lds(s->d, 1, true);
  p.nrowclass = s->nrowclass;
  for (int k = 0; k < mjx::kRowClasses; k++) p.row_cap[k] = s->row_cap[k];
  p.gscr = s->gscr;
  p.wl_list = s->wl;
  p.wl_seg = s->wl ? s->wl + s->nworld : nullptr;
  p.gC = s->gC;
  p.gF = s->gF;
  p.gstride = s->gstride;
  p.spec = s->spec;
  p.nair = s->nair;
  for (int i = 0; i < mjx::kMaxAirSlots; i++) p.air_found[i] = s->air_found[i];
  p.air_cur = s->air_buf[0]; p.air_last = s->air_buf[1]; p.air_cc = s->air_buf[2];
  p.air_lc = s->air_buf[3]; p.air_time = s->air_buf[4];
  static const int minrows = [] {
    const char* e = getenv("MJX355_STAMP_MINROWS");
    return e ? atoi(e) : 0;
  }();
  p.stamp_minrows = minrows;
  static const int outputs_every = [] {
    const char* e = getenv("MJX355_OUTPUTS_EVERY");
    return e ? atoi(e) : 0;
  }();
  p.outputs_every = outputs_every;
  p.ovf_resolve = s->big ? 1 : 0;
  p.ovf_cap = s->ovf_cap;
  p.ovf_list = s->ovf;
  p.ovf_n = s->ovf ? s->ovf + (size_t)mjx::kMaxSplit * 2 * s->ovf_cap : nullptr;
  p.ovf_flag = s->ovf ? p.ovf_n + mjx::kMaxSplit * 2 : nullptr;
  p.ovf_done = s->ovf ? p.ovf_flag + s->nworld : nullptr;
  p.con_stride = s->con_stride;
  return p;
}

// The max-capacity launch parameters of the overflow re-solve: same model, data, lists and
// air-time buffers; the max dims, carves, kernels and scratch; no row classes (its worlds run
// the latency Newton kernel); overflow past it drops contacts.
static mjx::Params host_params_big(const mjxSim_* s) {
  mjx::Params p = host_params(s);
  p.d = s->dbig;
  for (int i = 0; i < 3; i++) p.LP[i] = s->lds_big[i];
  for (int k = 0; k < mjx::kRowClasses; k++) p.LP[3 + k] = s->lds_big[1];
  p.LPJ = mjx::make_lds(s->dbig, 1, true);
  p.nrowclass = 0;
  p.gscr = s->gscr_big;
  p.gC = s->gC_big;
  p.gF = s->gF_big;
  p.gstride = s->gstride_big;
  p.spec = s->spec_big;
  p.ovf_resolve = 0;
  return p;
}

// Upload the launch parameters (stream-ordered, so later launches see the new copy).
static int sync_params(mjxSim_* s, void* stream) {
  static thread_local mjx::Params staging, staging_big;
  staging = host_params(s);
  HIPCHK(hipMemcpyAsync(s->dparams, &staging, sizeof(mjx::Params), hipMemcpyHostToDevice,
                        (hipStream_t)stream));
  if (s->big) {
    staging_big = host_params_big(s);
    HIPCHK(hipMemcpyAsync(s->dparams_big, &staging_big, sizeof(mjx::Params), hipMemcpyHostToDevice,
                          (hipStream_t)stream));
  }
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

extern "C" {

const char* mjx_last_error(void) { return g_err.c_str(); }
int mjx_abi_version(void) { return MJX_ABI_VERSION; }
size_t mjx_model_desc_size(void) { return sizeof(mjxModelDesc); }

int mjx_model_create(const mjxModelDesc* desc, int device, mjxModel** out) {
  if (!desc || !out) return fail("null argument");
  if (desc->abi_version != MJX_ABI_VERSION) return fail("ABI version mismatch");
  if (desc->nbody > mjx::kMaxBodies) return fail("at most 64 bodies per world supported");
  if (desc->nv > mjx::kMaxDof) return fail("at most 64 dofs per world supported");
  if (desc->nu > mjx::kMaxLanes || desc->njnt > mjx::kMaxLanes)
    return fail("at most 64 actuators and 64 joints per world supported");
  if (desc->cone != 0) return fail("only pyramidal cones are supported");
  if (desc->contact_maxmatch < 1) return fail("contact_maxmatch must be >= 1");
  HIPCHK(hipSetDevice(device));
  auto* m = new mjxModel_();
  m->device = device;
  mjx::Dims& d = m->d;
  d.nq = desc->nq; d.nv = desc->nv; d.nu = desc->nu; d.nbody = desc->nbody; d.njnt = desc->njnt;
  d.ngeom = desc->ngeom; d.nsite = desc->nsite; d.nsensor = desc->nsensor;
  d.nsensordata = desc->nsensordata; d.npair = desc->npair; d.nhfield = desc->nhfield;
  d.nhfielddata = desc->nhfielddata; d.nlevel = desc->nlevel;
  d.nchild = desc->body_childadr[desc->nbody];
  if (d.nchild < 1) d.nchild = 1;
  d.nmocap = 0;
  for (int b = 0; b < d.nbody; b++)
    if (desc->body_mocapid[b] >= 0) d.nmocap++;
  d.nconmax = 0; d.njmax = 0;
  mjx::Opt& o = m->o;
  o.timestep = (float)desc->timestep; o.tolerance = (float)desc->tolerance;
  o.ls_tolerance = (float)desc->ls_tolerance; o.impratio = (float)desc->impratio;
  o.meaninertia = (float)desc->meaninertia;
  for (int i = 0; i < 3; i++) o.gravity[i] = (float)desc->gravity[i];
  o.iterations = desc->iterations; o.ls_iterations = desc->ls_iterations;
  o.integrator = desc->integrator; o.cone = desc->cone;
  o.maxmatch = desc->contact_maxmatch;

  auto upload = [&](const void* src, size_t bytes, void** dst) -> int {
    size_t nb = bytes > 0 ? bytes : 4;
    HIPCHK(hipMalloc(dst, nb));
    m->allocs.push_back(*dst);
    if (bytes > 0) HIPCHK(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    else HIPCHK(hipMemset(*dst, 0, nb));
    return 0;
  };
#define X_INT(name, cnt, w)                                                              \
  {                                                                                      \
    size_t n_ = (size_t)(cnt) * (w);                                                     \
    void* p_ = nullptr;                                                                  \
    if (upload(desc->name, n_ * sizeof(int32_t), &p_)) { delete m; return -1; }         \
    m->dm.name = (const int32_t*)p_;                                                     \
    m->int_dims[#name] = {(int64_t)(cnt), (int64_t)(w)};                                 \
  }
#define X_FLT(name, cnt, w)                                                              \
  {                                                                                      \
    size_t n_ = (size_t)(cnt) * (w);                                                     \
    std::vector<float> h_(n_);                                                           \
    for (size_t i = 0; i < n_; i++) h_[i] = (float)desc->name[i];                        \
    void* p_ = nullptr;                                                                  \
    if (upload(h_.data(), n_ * sizeof(float), &p_)) { delete m; return -1; }            \
    m->dm.name = (const float*)p_;                                                       \
    m->dm.name##_ws = 0;                                                                 \
    m->host_float[#name] = std::move(h_);                                                \
    m->float_dims[#name] = {(int64_t)(cnt), (int64_t)(w)};                               \
  }
  MJX_MODEL_INT_FIELDS(X_INT)
  MJX_MODEL_FLOAT_FIELDS(X_FLT)
#undef X_INT
#undef X_FLT
  void* p = nullptr;
  if (upload(desc->dof_bodymask, sizeof(uint64_t) * d.nv, &p)) { delete m; return -1; }
  m->dm.dof_bodymask = (const uint64_t*)p;
  {
    m->dof_parentid.assign(desc->dof_parentid, desc->dof_parentid + d.nv);
    // ancestor masks along dof_parentid (parents precede children in dof order)
    std::vector<uint64_t> anc(d.nv > 0 ? d.nv : 1, 0);
    for (int i = 0; i < d.nv; i++) {
      const int par = desc->dof_parentid[i];
      anc[i] = (1ull << i) | (par >= 0 && par < i ? anc[par] : 0ull);
    }
    if (upload(anc.data(), sizeof(uint64_t) * anc.size(), &p)) { delete m; return -1; }
    m->dm.dof_ancmask = (const uint64_t*)p;
    // subtree masks (parents precede children in body order) and the dofs moving each body
    const int nb = d.nbody;
    std::vector<uint64_t> sub(nb > 0 ? nb : 1, 0), bdof(nb > 0 ? nb : 1, 0);
    for (int b = nb - 1; b >= 0; b--) {
      sub[b] |= 1ull << b;
      const int par = desc->body_parentid[b];
      if (b > 0 && par >= 0 && par < b) sub[par] |= sub[b];
    }
    for (int b = 0; b < nb; b++) {
      const int par = desc->body_parentid[b];
      if (b > 0 && par >= 0 && par < b) bdof[b] = bdof[par];
      for (int k = 0; k < desc->body_dofnum[b]; k++) bdof[b] |= 1ull << (desc->body_dofadr[b] + k);
    }
    if (upload(sub.data(), sizeof(uint64_t) * sub.size(), &p)) { delete m; return -1; }
    m->dm.body_submask = (const uint64_t*)p;
    if (upload(bdof.data(), sizeof(uint64_t) * bdof.size(), &p)) { delete m; return -1; }
    m->dm.body_dofmask = (const uint64_t*)p;
    // per-lane records (engine.h DModel::body_rec): level-order bodies, dofs, actuators
    const int nlev = d.nlevel;
    std::vector<int32_t> brec((size_t)mjx::kBodyRec * (nb > 0 ? nb : 1), 0);
    for (int i = 0; i < nb; i++) {
      int32_t* r = brec.data() + (size_t)mjx::kBodyRec * i;
      const int b = desc->level_body[i];
      int lv = 0;
      for (int l = 1; l < nlev; l++) lv = i >= desc->level_start[l] ? l : lv;
      const int j0 = desc->body_jntadr[b], jn = desc->body_jntnum[b], k = jn > 0 ? j0 : 0;
      const int c0 = desc->body_childadr[b], cn = desc->body_childadr[b + 1] - c0;
      int chp = 0;
      for (int t = 0; t < 5 && t < cn; t++) chp |= desc->body_child[c0 + t] << (6 * t);
      const int32_t v[16] = {b, desc->body_parentid[b], lv, j0, jn, desc->jnt_type[k], desc->jnt_qposadr[k],
                             desc->jnt_dofadr[k], desc->body_dofadr[b], desc->body_dofnum[b],
                             desc->body_mocapid[b], desc->body_rootid[b], c0, cn, chp, 0};
      for (int t = 0; t < 16; t++) r[t] = v[t];
      r[16] = (int32_t)(uint32_t)sub[b]; r[17] = (int32_t)(uint32_t)(sub[b] >> 32);
      r[18] = (int32_t)(uint32_t)bdof[b]; r[19] = (int32_t)(uint32_t)(bdof[b] >> 32);
    }
    if (upload(brec.data(), sizeof(int32_t) * brec.size(), &p)) { delete m; return -1; }
    m->dm.body_rec = (const int32_t*)p;
    const int nv = d.nv;
    std::vector<int32_t> drec((size_t)mjx::kDofRec * (nv > 0 ? nv : 1), 0);
    for (int i = 0; i < nv; i++) {
      int32_t* r = drec.data() + (size_t)mjx::kDofRec * i;
      const int j = desc->dof_jntid[i], body = desc->dof_bodyid[i];
      const int32_t v[8] = {body, desc->jnt_type[j], desc->jnt_qposadr[j], desc->body_parentid[body],
                            desc->jnt_dofadr[j], desc->body_dofadr[body], j, 0};
      for (int t = 0; t < 8; t++) r[t] = v[t];
      r[8] = (int32_t)(uint32_t)anc[i]; r[9] = (int32_t)(uint32_t)(anc[i] >> 32);
    }
    if (upload(drec.data(), sizeof(int32_t) * drec.size(), &p)) { delete m; return -1; }
    m->dm.dof_rec = (const int32_t*)p;
    const int nu = d.nu;
    std::vector<int32_t> arec((size_t)mjx::kActRec * (nu > 0 ? nu : 1), 0);
    for (int u = 0; u < nu; u++) {
      int32_t* r = arec.data() + (size_t)mjx::kActRec * u;
      const int j = desc->actuator_trnid[u];
      r[0] = desc->jnt_dofadr[j]; r[1] = desc->jnt_qposadr[j];
      r[2] = desc->actuator_ctrllimited[u]; r[3] = desc->actuator_forcelimited[u];
    }
    if (upload(arec.data(), sizeof(int32_t) * arec.size(), &p)) { delete m; return -1; }
    m->dm.act_rec = (const int32_t*)p;
  }
  {
    // Terrain broadphase tables.  The pair list is [regular pairs | terrain pairs], the
    // terrain pairs grouped by their static terrain geom (the scene compiler emits them that
    // way): a heightfield, or a box on a body welded to the world.  Those geoms keep no LDS
    // frame; their world frames and AABBs are static and derived here.
    const int ng = desc->ngeom, np = desc->npair;
    if (desc->nmaskword < (ng + 31) / 32) { delete m; return fail("nmaskword < ceil(ngeom / 32)"); }
    m->dm.nmaskword = desc->nmaskword;
    auto is_static = [&](int g) {
      const int t = desc->geom_type[g];
      return t == mjx::GEOM_HFIELD ||
             (t == mjx::GEOM_BOX && desc->body_weldid[desc->geom_bodyid[g]] == 0);
    };
    std::vector<int> geom_lds(ng > 0 ? ng : 1, -1), lds_geom;
    for (int g = 0; g < ng; g++)
      if (!is_static(g)) { geom_lds[g] = (int)lds_geom.size(); lds_geom.push_back(g); }
    d.ngeom_lds = (int)lds_geom.size();
    if (lds_geom.empty()) lds_geom.push_back(0);
    int nreg = 0;
    while (nreg < np && !is_static(desc->pair_geom1[nreg]) && !is_static(desc->pair_geom2[nreg])) nreg++;
    std::vector<int> st_geom, st_adr, partner;
    std::vector<char> seen(ng > 0 ? ng : 1, 0), done(ng > 0 ? ng : 1, 0);
    for (int q = nreg; q < np; q++) {
      const int g1 = desc->pair_geom1[q], g2 = desc->pair_geom2[q];
      if (is_static(g1) == is_static(g2)) {
        delete m;
        return fail("pair list: terrain pairs (one static terrain geom each) must follow all regular pairs");
      }
      const int sg = is_static(g1) ? g1 : g2, pg = is_static(g1) ? g2 : g1;
      if (desc->geom_type[sg] == mjx::GEOM_HFIELD ? sg != g1
                                                  : (sg != g2 && desc->geom_type[pg] != mjx::GEOM_BOX)) {
        delete m;
        return fail("pair list: a terrain pair must keep MuJoCo's geom-type order");
      }
      if (st_geom.empty() || st_geom.back() != sg) {
        if (done[sg]) { delete m; return fail("pair list: terrain pair blocks must be contiguous"); }
        done[sg] = 1;
        st_geom.push_back(sg);
        st_adr.push_back(q);
      }
      if (!seen[pg]) { seen[pg] = 1; partner.push_back(pg); }
    }
    st_adr.push_back(np);
    d.npair = nreg;
    d.npair_all = np;
    d.nboxbox = 0;
    for (int q = 0; q < np; q++)
      d.nboxbox += desc->geom_type[desc->pair_geom1[q]] == mjx::GEOM_BOX &&
                   desc->geom_type[desc->pair_geom2[q]] == mjx::GEOM_BOX;
    d.nstatic = (int)st_geom.size();
    d.nstpartner = (int)partner.size();
    // static world frames of the terrain geoms (D.geom_xpos / geom_xmat, AABBs)
    std::vector<float> aabb((size_t)6 * std::max((int)st_geom.size(), 1), 0.f);
    std::vector<int> st_slot(ng > 0 ? ng : 1, -1);
    for (size_t k = 0; k < st_geom.size(); k++) st_slot[st_geom[k]] = (int)k;
    for (int g = 0; g < ng; g++) {
      if (!is_static(g)) continue;
      int b = desc->geom_bodyid[g];
      if (desc->body_weldid[b] != 0) {
        delete m;
        return fail("heightfield geoms must sit on bodies welded to the world");
      }
      // chain of static bodies up to the world: x = x_parent + R_parent p, q = q_parent q
      double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, x[3] = {0, 0, 0};
      std::vector<int> chain;
      for (int c = b; c > 0; c = desc->body_parentid[c]) chain.push_back(c);
      auto qm = [](const double* q, double* M) {
        const double w = q[0], a = q[1], bq = q[2], c = q[3];
        M[0] = 1 - 2 * (bq * bq + c * c); M[1] = 2 * (a * bq - w * c); M[2] = 2 * (a * c + w * bq);
        M[3] = 2 * (a * bq + w * c); M[4] = 1 - 2 * (a * a + c * c); M[5] = 2 * (bq * c - w * a);
        M[6] = 2 * (a * c - w * bq); M[7] = 2 * (bq * c + w * a); M[8] = 1 - 2 * (a * a + bq * bq);
      };
      auto step = [&](const double* pos, const double* quat) {
        double Q[9], nx[3], nR[9];
        qm(quat, Q);
        for (int i = 0; i < 3; i++) nx[i] = x[i] + R[3 * i] * pos[0] + R[3 * i + 1] * pos[1] + R[3 * i + 2] * pos[2];
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++)
            nR[3 * i + j] = R[3 * i] * Q[j] + R[3 * i + 1] * Q[3 + j] + R[3 * i + 2] * Q[6 + j];
        for (int i = 0; i < 3; i++) x[i] = nx[i];
        for (int i = 0; i < 9; i++) R[i] = nR[i];
      };
      for (auto it = chain.rbegin(); it != chain.rend(); ++it)
        step(desc->body_pos + 3 * *it, desc->body_quat + 4 * *it);
      step(desc->geom_pos + 3 * g, desc->geom_quat + 4 * g);
      m->static_geoms.push_back(g);
      for (int i = 0; i < 3; i++) m->static_xpos.push_back((float)x[i]);
      for (int i = 0; i < 9; i++) m->static_xmat.push_back((float)R[i]);
      const int k = st_slot[g];
      if (k < 0) continue;
      // local box: a box's half sizes; a heightfield's [-sx, sx] x [-sy, sy] x [-base, zmax]
      double e[3], c[3] = {0, 0, 0};
      if (desc->geom_type[g] == mjx::GEOM_BOX) {
        for (int i = 0; i < 3; i++) e[i] = desc->geom_size[3 * g + i];
      } else {
        const double* hs = desc->hfield_size + 4 * desc->geom_dataid[g];
        e[0] = hs[0]; e[1] = hs[1]; e[2] = 0.5 * (hs[2] + hs[3]);
        c[2] = 0.5 * (hs[2] - hs[3]);
      }
      const double mg = desc->geom_margin[g];
      for (int i = 0; i < 3; i++) {
        const double cw = x[i] + R[3 * i] * c[0] + R[3 * i + 1] * c[1] + R[3 * i + 2] * c[2];
        const double hw = std::fabs(R[3 * i]) * e[0] + std::fabs(R[3 * i + 1]) * e[1] +
                          std::fabs(R[3 * i + 2]) * e[2] + mg;
        // rounded outward so the fp32 cull never rejects what the fp64 bounds admit
        aabb[6 * k + i] = std::nextafter((float)(cw - hw), -INFINITY);
        aabb[6 * k + 3 + i] = std::nextafter((float)(cw + hw), INFINITY);
      }
    }
    const int nchunk = std::max(1, (d.nstatic + mjx::kStaticChunk - 1) / mjx::kStaticChunk);
    std::vector<float> chunk((size_t)6 * nchunk);
    for (int c = 0; c < nchunk; c++) {
      float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int k = c * mjx::kStaticChunk; k < std::min(d.nstatic, (c + 1) * mjx::kStaticChunk); k++)
        for (int i = 0; i < 3; i++) {
          lo[i] = std::min(lo[i], aabb[6 * k + i]);
          hi[i] = std::max(hi[i], aabb[6 * k + 3 + i]);
        }
      for (int i = 0; i < 3; i++) { chunk[6 * c + i] = lo[i]; chunk[6 * c + 3 + i] = hi[i]; }
    }
    if (st_geom.empty()) { st_geom.push_back(0); partner.push_back(0); }
    if (upload(geom_lds.data(), sizeof(int) * geom_lds.size(), &p)) { delete m; return -1; }
    m->dm.geom_lds = (const int32_t*)p;
    if (upload(lds_geom.data(), sizeof(int) * lds_geom.size(), &p)) { delete m; return -1; }
    m->dm.lds_geom = (const int32_t*)p;
    if (upload(st_geom.data(), sizeof(int) * st_geom.size(), &p)) { delete m; return -1; }
    m->dm.st_geom = (const int32_t*)p;
    if (upload(st_adr.data(), sizeof(int) * st_adr.size(), &p)) { delete m; return -1; }
    m->dm.st_pairadr = (const int32_t*)p;
    if (upload(partner.data(), sizeof(int) * partner.size(), &p)) { delete m; return -1; }
    m->dm.st_partner = (const int32_t*)p;
    if (upload(aabb.data(), sizeof(float) * aabb.size(), &p)) { delete m; return -1; }
    m->dm.st_aabb = (const float*)p;
    if (upload(chunk.data(), sizeof(float) * chunk.size(), &p)) { delete m; return -1; }
    m->dm.st_chunk_aabb = (const float*)p;
    // regular-pair records: the pair loop of phase A reads one coalesced 16-B record per
    // lane instead of a chain of dependent per-geom loads (pair -> geom -> type / slot /
    // margin / rbound); the cull radius is formed in fp32 exactly as the kernel forms it
    bool packable = ng < 65536 && d.ngeom_lds < 4096;
    for (int g = 0; g < ng && packable; g++) packable = desc->geom_type[g] >= 0 && desc->geom_type[g] < 16;
    m->dm.pair_rec = nullptr;
    if (packable && nreg > 0) {
      std::vector<int32_t> rec((size_t)4 * nreg);
      for (int q = 0; q < nreg; q++) {
        const int g1 = desc->pair_geom1[q], g2 = desc->pair_geom2[q];
        const int t1 = desc->geom_type[g1], t2 = desc->geom_type[g2];
        const float r1 = (float)desc->geom_rbound[g1], r2 = (float)desc->geom_rbound[g2];
        const float mg = std::fmax((float)desc->geom_margin[g1], (float)desc->geom_margin[g2]);
        const float cull = (r1 > 0 && r2 > 0 && t1 != mjx::GEOM_HFIELD) ? r1 + r2 + mg : INFINITY;
        rec[4 * q] = g1 | g2 << 16;
        rec[4 * q + 1] = geom_lds[g1] | geom_lds[g2] << 12 | t1 << 24 | (int32_t)((uint32_t)t2 << 28);
        std::memcpy(&rec[4 * q + 2], &mg, 4);
        std::memcpy(&rec[4 * q + 3], &cull, 4);
      }
      if (upload(rec.data(), sizeof(int32_t) * rec.size(), &p)) { delete m; return -1; }
      m->dm.pair_rec = (const int32_t*)p;
    }
  }
  if (upload(desc->sensor_geommask1, sizeof(uint32_t) * (size_t)desc->nmaskword * d.nsensor, &p)) { delete m; return -1; }
  m->dm.sensor_geommask1 = (const uint32_t*)p;
  if (upload(desc->sensor_geommask2, sizeof(uint32_t) * (size_t)desc->nmaskword * d.nsensor, &p)) { delete m; return -1; }
  m->dm.sensor_geommask2 = (const uint32_t*)p;
  {
    // transposed single-slot contact-sensor masks (engine.h geom_csmask1/2); more than 64
    // such sensors: ncsens = 0 and phase C matches sensor by sensor (serial path)
    std::vector<int32_t> cs;
    for (int s = 0; s < d.nsensor; s++)
      if (desc->sensor_type[s] == mjx::SENS_CONTACT && desc->sensor_intprm[3 * s + 2] <= 1) cs.push_back(s);
    const int ng = std::max(d.ngeom, 1);
    std::vector<uint64_t> g1(ng, 0), g2(ng, 0);
    if (cs.size() <= 64) {
      for (size_t k = 0; k < cs.size(); k++) {
        const uint32_t* a = desc->sensor_geommask1 + (size_t)desc->nmaskword * cs[k];
        const uint32_t* b = desc->sensor_geommask2 + (size_t)desc->nmaskword * cs[k];
        for (int g = 0; g < d.ngeom; g++) {
          if ((a[g >> 5] >> (g & 31)) & 1u) g1[g] |= 1ull << k;
          if ((b[g >> 5] >> (g & 31)) & 1u) g2[g] |= 1ull << k;
        }
      }
      m->dm.ncsens = (int)cs.size();
    } else {
      m->dm.ncsens = 0;
    }
    if (cs.empty()) cs.push_back(0);
    if (upload(cs.data(), sizeof(int32_t) * cs.size(), &p)) { delete m; return -1; }
    m->dm.cs_sensor = (const int32_t*)p;
    if (upload(g1.data(), sizeof(uint64_t) * g1.size(), &p)) { delete m; return -1; }
    m->dm.geom_csmask1 = (const uint64_t*)p;
    if (upload(g2.data(), sizeof(uint64_t) * g2.size(), &p)) { delete m; return -1; }
    m->dm.geom_csmask2 = (const uint64_t*)p;
  }
  *out = m;
  return 0;
}

int mjx_model_destroy(mjxModel* m) {
  if (!m) return 0;
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
  return 0;
}

int mjx_sim_create(const mjxModel* model, int nworld, int nconmax, int njmax, mjxSim** out) {
  return mjx_sim_create_ex(model, nworld, nconmax, njmax, nconmax, njmax, out);
}

int mjx_sim_create_ex(const mjxModel* model, int nworld, int nconmax, int njmax,
                      int nconmax_max, int njmax_max, mjxSim** out) {
  if (!model || !out) return fail("null argument");
  if (nworld <= 0) return fail("nworld must be positive");
  if (nconmax <= 0 || nconmax > mjx::kWave)
    return fail("nconmax (contacts held per world) must be in [1, 64]");
  if (njmax <= 0) return fail("njmax must be positive");
  if (nconmax_max < nconmax || nconmax_max > mjx::kMaxContacts || njmax_max < njmax)
    return fail("max capacity: nconmax <= nconmax_max <= 512 and njmax <= njmax_max");
  if (nconmax_max > mjx::kWave && nconmax_max > njmax_max)
    return fail("a max capacity past 64 contacts needs njmax_max >= nconmax_max (the contact sort's "
                "scratch is the row block)");
  HIPCHK(hipSetDevice(model->device));
  auto* s = new mjxSim_();
  s->model = model;
  s->nworld = nworld;
  s->d = model->d;
  s->d.nconmax = nconmax;
  s->d.njmax = njmax;
  s->dm = model->dm;
  for (int i = 0; i < 3; i++) {
    s->lds_ph[i] = mjx::make_lds(s->d, i);
    if ((size_t)s->lds_ph[i].total * 4 > 160 * 1024) {
      delete s;
      return fail("per-world LDS footprint exceeds 160 KiB; lower njmax/nconmax");
    }
  }
  s->spec = mjx::find_spec(s->d, model->dof_parentid.data());
  s->nrowclass = mjx::choose_row_classes(s->d, s->spec, s->row_cap);
  // batch splits (launch_step): large batches of models without row classes run as
  // concurrent halves.  MJX355_SPLIT=<n> overrides (diagnostic; 1 = one launch set per phase),
  // also for models with row classes (each split then forks its own class streams).
  s->side.nsplit = nworld >= mjx::kSplitMinWorlds && s->nrowclass == 0 ? 2 : 1;
  if (const char* ev = getenv("MJX355_SPLIT")) s->side.nsplit = std::max(1, std::min(atoi(ev), mjx::kMaxSplit));
  // The overflow re-solve forks its chain from the stream that ran phase A.  With batch
  // splits that is a split stream, and a second-level fork from a captured side stream
  // crashes hipStreamEndCapture under the HIP runtime torch bundles:
  // split batches without row classes run the chain in line on their split stream instead
  // (launch_step); split batches with row classes (a diagnostic topology) keep the fast
  // carve as their max capacity (overflow drops, counted).
  s->big = (nconmax_max > nconmax || njmax_max > njmax) &&
           (s->side.nsplit == 1 || s->nrowclass == 0);
  s->con_stride = s->big ? nconmax_max : nconmax;
  if (s->big) {
    s->dbig = s->d;
    s->dbig.nconmax = nconmax_max;
    s->dbig.njmax = njmax_max;
    for (int i = 0; i < 3; i++) {
      s->lds_big[i] = mjx::make_lds(s->dbig, i);
      if ((size_t)s->lds_big[i].total * 4 > 160 * 1024) {
        delete s;
        return fail("max-capacity LDS footprint exceeds 160 KiB; lower njmax_max/nconmax_max");
      }
    }
    s->spec_big = mjx::find_spec(s->dbig, model->dof_parentid.data());
    s->gC_big = (s->lds_big[1].pack_len + 63) & ~63;
    s->gF_big = s->gC_big + ((s->lds_big[2].pack_len + 63) & ~63);
    s->gstride_big = s->gF_big + ((mjx::ltr_size((s->d.nv + 3) & ~3) + 63) & ~63);
    // re-solve list capacity per split and substep parity: every world may be listed
    s->ovf_cap = nworld;
  }
  for (int k = 0; k < mjx::kRowClasses; k++) {
    mjx::Dims ds = s->d;
    ds.njmax = k < s->nrowclass ? s->row_cap[k] : s->d.njmax;
    s->lds_ph[3 + k] = mjx::make_lds(ds, 1);
  }
  {
    hipError_t e = hipSuccess;
    if (s->side.nsplit > 1) {
      e = hipEventCreateWithFlags(&s->side.split_fork, hipEventDisableTiming);
      for (int p = 1; p < s->side.nsplit && e == hipSuccess; p++) {
        e = hipStreamCreateWithFlags(&s->side.split[p], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s->side.split_join[p], hipEventDisableTiming);
      }
    }
    // default priority: measured, high-priority side streams let the few heavy worlds hold
    // LDS that the bulk of small-class worlds needs (Newton span 214 -> 281 us, G1 4096)
    for (int p = 0; p < s->side.nsplit && s->nrowclass > 0 && e == hipSuccess; p++) {
      e = hipEventCreateWithFlags(&s->side.fork[p], hipEventDisableTiming);
      for (int k = 0; k < s->nrowclass && e == hipSuccess; k++) {
        e = hipStreamCreateWithFlags(&s->side.stream[p][k], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s->side.join[p][k], hipEventDisableTiming);
      }
    }
    for (int p = 0; p < s->side.nsplit && s->big && e == hipSuccess; p++) {
      e = hipStreamCreateWithFlags(&s->side.ovf[p], hipStreamNonBlocking);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&s->side.ovf_fork[p], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&s->side.ovf_join[p], hipEventDisableTiming);
    }
    if (e != hipSuccess) { delete s; return fail(std::string("side streams: ") + hipGetErrorString(e)); }
  }
  s->gC = (s->lds_ph[1].pack_len + 63) & ~63;
  s->gF = s->gC + ((s->lds_ph[2].pack_len + 63) & ~63);
  {
    const int nvp = (s->d.nv + 3) & ~3;
    s->gstride = s->gF + ((mjx::ltr_size(nvp) + 63) & ~63);  // implicit factor, LTR form
  }
  // the contact output arrays hold the max capacity's contacts
  mjx::Dims dout = s->d;
  dout.nconmax = s->con_stride;
  const mjx::Dims& d = dout;
  // data arena: one allocation, 256-B aligned sub-buffers
  size_t off = 0;
  std::vector<std::pair<std::string, size_t>> offs;
  auto reserve = [&](const std::string& name, size_t bytes) {
    offs.push_back({name, off});
    off += (bytes + 255) & ~(size_t)255;
  };
#define X_FLT(name, cnt, w) reserve(#name, sizeof(float) * (size_t)nworld * (cnt) * (w));
#define X_INT(name, cnt, w) reserve(#name, sizeof(int32_t) * (size_t)nworld * (cnt) * (w));
  MJX_DATA_FLOAT_FIELDS(X_FLT)
  MJX_DATA_INT_FIELDS(X_INT)
#undef X_FLT
#undef X_INT
  reserve("__stats", sizeof(int32_t) * 8);
  reserve("__wstats", sizeof(int32_t) * 8 * (size_t)nworld);
  reserve("__evtotal", sizeof(int32_t) * 4);
  reserve("__prof", sizeof(unsigned long long) * 48);
  reserve("__wtrace", sizeof(unsigned long long) * 8 * (size_t)nworld);
  hipError_t e = hipMalloc((void**)&s->gscr, sizeof(float) * (size_t)nworld * s->gstride);
  if (e != hipSuccess) { delete s; return fail(std::string("hipMalloc scratch: ") + hipGetErrorString(e)); }
  e = hipMemset(s->gscr, 0, sizeof(float) * (size_t)nworld * s->gstride);
  if (e != hipSuccess) { delete s; return fail(std::string("hipMemset: ") + hipGetErrorString(e)); }
  e = hipMalloc((void**)&s->wl, sizeof(int) * ((size_t)nworld + 2 * (mjx::kRowClasses + 1) * mjx::kMaxSplit));
  if (e != hipSuccess) { delete s; return fail(std::string("hipMalloc work lists: ") + hipGetErrorString(e)); }
  e = hipMemset(s->wl, 0, sizeof(int) * ((size_t)nworld + 2 * (mjx::kRowClasses + 1) * mjx::kMaxSplit));
  if (e != hipSuccess) { delete s; return fail(std::string("hipMemset: ") + hipGetErrorString(e)); }
  if (s->big) {
    const size_t gb = sizeof(float) * (size_t)nworld * s->gstride_big;
    e = hipMalloc((void**)&s->gscr_big, gb);
    if (e == hipSuccess) e = hipMemset(s->gscr_big, 0, gb);
    const size_t ob = sizeof(int) * ((size_t)mjx::kMaxSplit * 2 * (s->ovf_cap + 2) + nworld);
    if (e == hipSuccess) e = hipMalloc((void**)&s->ovf, ob);
    if (e == hipSuccess) e = hipMemset(s->ovf, 0, ob);
    if (e == hipSuccess) e = hipMalloc((void**)&s->dparams_big, sizeof(mjx::Params));
    if (e != hipSuccess) { delete s; return fail(std::string("hipMalloc re-solve buffers: ") + hipGetErrorString(e)); }
  }
  e = hipMalloc(&s->arena, off);
  if (e != hipSuccess) { delete s; return fail(std::string("hipMalloc data: ") + hipGetErrorString(e)); }
  e = hipMemset(s->arena, 0, off);
  if (e != hipSuccess) { delete s; return fail(std::string("hipMemset: ") + hipGetErrorString(e)); }
  size_t k = 0;
  char* base = (char*)s->arena;
  // a field whose count is the literal 1 (fields.h) is a per-world scalar; every other keeps
  // its count axis even when the model makes it 1 (qpos of a one-dof model is [nworld, 1])
#define X_FLT(name, cnt, w)                                                                  \
  s->dd.name = (float*)(base + offs[k++].second);                                            \
  s->fields[#name] = FieldInfo{s->dd.name, true, (int64_t)(cnt), (int64_t)(w), true, false,  \
                               std::string(#cnt) == "1"};                                    \
  s->names.push_back(#name);
#define X_INT(name, cnt, w)                                                                    \
  s->dd.name = (int32_t*)(base + offs[k++].second);                                            \
  s->fields[#name] = FieldInfo{s->dd.name, false, (int64_t)(cnt), (int64_t)(w), true, false,  \
                               std::string(#cnt) == "1"};                                      \
  s->names.push_back(#name);
  MJX_DATA_FLOAT_FIELDS(X_FLT)
  MJX_DATA_INT_FIELDS(X_INT)
#undef X_FLT
#undef X_INT
  // an unused contact slot holds geoms (-1, -1), as the outputs leave every slot past ncon
  // (a slot never written must read the same as one cleared: fused and single steps write
  // outputs on different substeps)
  e = hipMemset(s->dd.contact_geom, 0xff, sizeof(int32_t) * (size_t)nworld * d.nconmax * 2);
  if (e != hipSuccess) { delete s; return fail(std::string("hipMemset: ") + hipGetErrorString(e)); }
  s->dd.stats = (int32_t*)(base + offs[k++].second);
  s->dd.wstats = (int32_t*)(base + offs[k++].second);
  // per-world engine counters [nworld, 8] (phase C, last substep): [0] contacts found,
  // [1] rows, [2] contact-overflow / [3] row-overflow / [4] unsupported-pair events
  // (cumulative), [5] Newton iterations -- a zero-copy view for device-side logging
  s->fields["engine_counters"] = FieldInfo{s->dd.wstats, false, 8, 1, true, false};
  s->names.push_back("engine_counters");
  // [1, 4]: contact-overflow / row-overflow / unsupported-pair events summed over worlds
  s->dd.evtotal = (int32_t*)(base + offs[k++].second);
  s->fields["engine_events"] = FieldInfo{s->dd.evtotal, false, 4, 1, false, false};
  s->names.push_back("engine_events");
  s->dd.prof = (unsigned long long*)(base + offs[k++].second);
  // per-world phase start/end timestamps (s_memrealtime, 100 MHz; diagnostic MJX_STAMPS
  // build): [A0 A1 B0 B1 C0 C1 - -] as int32 pairs
  s->dd.wtrace = (unsigned long long*)(base + offs[k++].second);
  s->fields["world_trace"] = FieldInfo{s->dd.wtrace, false, 16, 1, true, false};
  s->names.push_back("world_trace");
  s->stats = s->dd.stats;
  // model fields visible as "model.<name>"
  for (auto& kv : model->float_dims) {
    FieldInfo fi{nullptr, true, kv.second.first, kv.second.second, false, true};
    s->fields["model." + kv.first] = fi;
    s->names.push_back("model." + kv.first);
  }
  for (auto& kv : model->int_dims) {
    FieldInfo fi{nullptr, false, kv.second.first, kv.second.second, false, true};
    s->fields["model." + kv.first] = fi;
    s->names.push_back("model." + kv.first);
  }
  e = hipMalloc((void**)&s->dparams, sizeof(mjx::Params));
  if (e != hipSuccess) { delete s; return fail(std::string("hipMalloc params: ") + hipGetErrorString(e)); }
  if (sync_params(s, nullptr)) { delete s; return -1; }
  e = mjx::prepare_step(host_params(s));
  if (e == hipSuccess && s->big) e = mjx::prepare_step(host_params_big(s));
  s->side.range_chain = s->nrowclass == 0 && mjx::range_chain_default(host_params(s), nworld, s->side.nsplit);
  if (e != hipSuccess) { delete s; return fail(std::string("prepare: ") + hipGetErrorString(e)); }
  // heightfield geom frames are static: write them once for every world
  for (size_t k = 0; k < model->static_geoms.size(); k++) {
    const int g = model->static_geoms[k];
    std::vector<float> px((size_t)nworld * 3), pm((size_t)nworld * 9);
    for (int w = 0; w < nworld; w++) {
      for (int i = 0; i < 3; i++) px[(size_t)w * 3 + i] = model->static_xpos[3 * k + i];
      for (int i = 0; i < 9; i++) pm[(size_t)w * 9 + i] = model->static_xmat[9 * k + i];
    }
    e = hipMemcpy2D(s->dd.geom_xpos + 3 * g, sizeof(float) * 3 * d.ngeom, px.data(),
                    sizeof(float) * 3, sizeof(float) * 3, nworld, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy2D(s->dd.geom_xmat + 9 * g, sizeof(float) * 9 * d.ngeom, pm.data(),
                      sizeof(float) * 9, sizeof(float) * 9, nworld, hipMemcpyHostToDevice);
    if (e != hipSuccess) { delete s; return fail(std::string("hfield frames: ") + hipGetErrorString(e)); }
  }
  // initial state: mj_resetData
  if (mjx::launch_reset(d, s->dm, s->dd, nullptr, nworld, s->con_stride, nullptr) != hipSuccess) {
    delete s;
    return fail("reset launch failed");
  }
  e = hipDeviceSynchronize();
  if (e != hipSuccess) { delete s; return fail(std::string("sync: ") + hipGetErrorString(e)); }
  *out = s;
  return 0;
}

int mjx_sim_destroy(mjxSim* s) {
  if (!s) return 0;
  if (s->arena) (void)hipFree(s->arena);
  if (s->gscr) (void)hipFree(s->gscr);
  if (s->wl) (void)hipFree(s->wl);
  if (s->dparams) (void)hipFree(s->dparams);
  if (s->gscr_big) (void)hipFree(s->gscr_big);
  if (s->ovf) (void)hipFree(s->ovf);
  if (s->dparams_big) (void)hipFree(s->dparams_big);
  for (void* p : s->expanded_allocs) (void)hipFree(p);
  delete s;
  return 0;
}

int mjx_step(mjxSim* s, int nsubstep, void* stream) {
  if (!s) return fail("null sim");
  if (nsubstep < 1) return fail("nsubstep must be >= 1");
  const mjx::Params hb = s->big ? host_params_big(s) : mjx::Params{};
  hipError_t e = mjx::launch_step(host_params(s), s->dparams, s->nworld, nsubstep, 1, nullptr,
                                  (hipStream_t)stream, &s->side, s->big ? &hb : nullptr,
                                  s->dparams_big);
  if (e != hipSuccess) return fail(std::string("step launch: ") + hipGetErrorString(e));
  return 0;
}

int mjx_forward(mjxSim* s, void* stream) { return mjx_forward_masked(s, nullptr, stream); }

int mjx_forward_masked(mjxSim* s, const uint8_t* mask, void* stream) {
  if (!s) return fail("null sim");
  const mjx::Params hb = s->big ? host_params_big(s) : mjx::Params{};
  hipError_t e = mjx::launch_step(host_params(s), s->dparams, s->nworld, 1, 0, mask,
                                  (hipStream_t)stream, &s->side, s->big ? &hb : nullptr,
                                  s->dparams_big);
  if (e != hipSuccess) return fail(std::string("forward launch: ") + hipGetErrorString(e));
  return 0;
}

int mjx_sim_track_air_time(mjxSim* s, int n, const int32_t* found_adr, float* cur_air,
                           float* last_air, float* cur_contact, float* last_contact,
                           float* last_time, void* stream) {
  if (!s) return fail("null sim");
  if (n < 0 || n > mjx::kMaxAirSlots) return fail("air-time tracking: 0 <= n <= 8 slots");
  if (n > 0 && (!found_adr || !cur_air || !last_air || !cur_contact || !last_contact || !last_time))
    return fail("air-time tracking: null buffer");
  for (int i = 0; i < n; i++)
    if (found_adr[i] < 0 || found_adr[i] >= s->d.nsensordata)
      return fail("air-time tracking: found address outside sensordata");
  s->nair = n;
  for (int i = 0; i < mjx::kMaxAirSlots; i++) s->air_found[i] = i < n ? found_adr[i] : 0;
  float* b[5] = {cur_air, last_air, cur_contact, last_contact, last_time};
  for (int i = 0; i < 5; i++) s->air_buf[i] = n > 0 ? b[i] : nullptr;
  return sync_params(s, stream);
}

int mjx_reset(mjxSim* s, const uint8_t* mask, void* stream) {
  if (!s) return fail("null sim");
  hipError_t e = mjx::launch_reset(s->d, s->dm, s->dd, mask, s->nworld, s->con_stride, (hipStream_t)stream);
  if (e != hipSuccess) return fail(std::string("reset launch: ") + hipGetErrorString(e));
  return 0;
}

static void dl_deleter(DLManagedTensor* t) {
  if (!t) return;
  delete[] t->dl_tensor.shape;
  delete t;
}

static const void* model_field_ptr(const mjxSim_* s, const std::string& name, int* ws) {
  *ws = 0;
#define X_FLT(n, cnt, w) if (name == #n) { *ws = s->dm.n##_ws; return s->dm.n; }
#define X_INT(n, cnt, w) if (name == #n) { return s->dm.n; }
  MJX_MODEL_FLOAT_FIELDS(X_FLT)
  MJX_MODEL_INT_FIELDS(X_INT)
#undef X_FLT
#undef X_INT
  return nullptr;
}

int mjx_field(mjxSim* s, const char* cname, DLManagedTensor** out) {
  if (!s || !cname || !out) return fail("null argument");
  std::string name(cname);
  auto it = s->fields.find(name);
  if (it == s->fields.end()) return fail("unknown field '" + name + "'");
  const FieldInfo& fi = it->second;
  void* ptr = fi.ptr;
  int64_t lead = fi.per_world ? s->nworld : 1;
  if (fi.model) {
    int ws = 0;
    ptr = const_cast<void*>(model_field_ptr(s, name.substr(6), &ws));
    lead = ws > 0 ? s->nworld : 1;
  }
  auto* t = new DLManagedTensor();
  std::vector<int64_t> shape;
  shape.push_back(lead);
  if (!fi.scalar) shape.push_back(fi.count);
  if (fi.width > 1) shape.push_back(fi.width);
  t->dl_tensor.data = ptr;
  t->dl_tensor.device = DLDevice{kDLROCM, s->model->device};
  t->dl_tensor.ndim = (int32_t)shape.size();
  t->dl_tensor.dtype = fi.is_float ? DLDataType{2, 32, 1} : DLDataType{0, 32, 1};
  t->dl_tensor.shape = new int64_t[shape.size()];
  for (size_t i = 0; i < shape.size(); i++) t->dl_tensor.shape[i] = shape[i];
  t->dl_tensor.strides = nullptr;  // compact row-major
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = nullptr;
  t->deleter = dl_deleter;
  *out = t;
  return 0;
}

int mjx_field_count(const mjxSim* s) { return s ? (int)s->names.size() : 0; }
const char* mjx_field_name(const mjxSim* s, int i) {
  if (!s || i < 0 || i >= (int)s->names.size()) return nullptr;
  return s->names[i].c_str();
}

int mjx_field_is_expanded(const mjxSim* s, const char* cname) {
  if (!s || !cname) return 0;
  int ws = 0;
  model_field_ptr(s, std::string(cname), &ws);
  return ws > 0;
}

int mjx_expand_field(mjxSim* s, const char* cname, void* stream) {
  if (!s || !cname) return fail("null argument");
  std::string name(cname);
  auto hit = s->model->host_float.find(name);
  if (hit == s->model->host_float.end())
    return fail("field '" + name + "' is not an expandable float model field");
  const std::vector<float>& h = hit->second;
  size_t per = h.size();
  float* buf = nullptr;
  size_t bytes = sizeof(float) * (per > 0 ? per : 1) * (size_t)s->nworld;
  HIPCHK(hipMalloc((void**)&buf, bytes));
  s->expanded_allocs.push_back(buf);
  // tile the CURRENT values (default model values) to every world
  int ws = 0;
  const float* cur = (const float*)model_field_ptr(s, name, &ws);
  if (ws > 0) return fail("field '" + name + "' already expanded");
  // world 0 from the model, then doubling copies of the filled prefix: ceil(log2 N) + 1
  // copies instead of one per world (8,192 copy dispatches for Go1 at sim creation)
  if (s->nworld > 0)
    HIPCHK(hipMemcpyAsync(buf, cur, sizeof(float) * per, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  for (size_t done = 1; done < (size_t)s->nworld;) {
    const size_t n = std::min(done, (size_t)s->nworld - done);
    HIPCHK(hipMemcpyAsync(buf + done * per, buf, sizeof(float) * per * n, hipMemcpyDeviceToDevice,
                          (hipStream_t)stream));
    done += n;
  }
#define X_FLT(n, cnt, w) if (name == #n) { s->dm.n = buf; s->dm.n##_ws = (int)per; }
  MJX_MODEL_FLOAT_FIELDS(X_FLT)
#undef X_FLT
  return sync_params(s, stream);
}

int mjx_sim_profile(mjxSim* s, uint64_t* out, void* stream) {
  if (!s || !out) return fail("null argument");
  HIPCHK(hipMemcpyAsync(out, s->dd.prof, sizeof(uint64_t) * 48, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int mjx_sim_spec(const mjxSim* s) { return s ? s->spec : -1; }

int mjx_spec_register(const char* path) {
  if (!path) return fail("null path");
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(std::string("dlopen: ") + dlerror());
  using AbiFn = int (*)(void);
  using DimsFn = void (*)(mjx::Dims*);
  using TreeFn = int (*)(int*, int);
  using KernFn = mjx::StepFnPtr (*)(int);
  auto abi = reinterpret_cast<AbiFn>(dlsym(h, "mjx_jit_abi"));
  auto dims = reinterpret_cast<DimsFn>(dlsym(h, "mjx_jit_dims"));
  auto tree = reinterpret_cast<TreeFn>(dlsym(h, "mjx_jit_tree"));
  auto kern = reinterpret_cast<KernFn>(dlsym(h, "mjx_jit_kernel"));
  if (!abi || !dims || !tree || !kern) return fail(std::string(path) + ": not a jit.hip library");
  if (abi() != (int)sizeof(mjx::Dims)) return fail(std::string(path) + ": Dims layout mismatch (stale build)");
  // the kernels read Params / Lds / DData through this library's layout: the JIT library must
  // come from the same kernel headers (csrc/Makefile MJX_HDR_HASH), else a stale cache entry or
  // a header edited after the last engine build would fault the device instead of failing here
  using HdrFn = unsigned long long (*)(void);
  auto hdr = reinterpret_cast<HdrFn>(dlsym(h, "mjx_jit_hdr"));
#ifdef MJX_HDR_HASH
  if (!hdr || hdr() != (unsigned long long)MJX_HDR_HASH)
    return fail(std::string(path) + ": built from other kernel headers than libmjx355.so (rebuild one of them)");
#else
  if (!hdr) return fail(std::string(path) + ": not a jit.hip library of this engine");
#endif
  mjx::Dims d{};
  dims(&d);
  int par[64];
  const int n = tree(par, 64);
  if (n < 0 || n > 64) return fail("bad dof tree in the jit library");
  return mjx::register_spec(d, par, n, kern);  // the library stays loaded for the process
}

int mjx_sim_mass_matrix(mjxSim* s, int big, float* out, void* stream) {
  if (!s || !out) return fail("null argument");
  if (big && !s->big) return fail("the sim has no max-capacity scratch");
  const int nvp = (s->d.nv + 3) & ~3;
  const size_t n = (size_t)mjx::ltr_size(nvp);
  const float* src = (big ? s->gscr_big : s->gscr) + (big ? s->lds_big[1].M : s->lds_ph[1].M);
  const size_t pitch = sizeof(float) * (size_t)(big ? s->gstride_big : s->gstride);
  HIPCHK(hipMemcpy2DAsync(out, sizeof(float) * n, src, pitch, sizeof(float) * n, s->nworld,
                          hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

int mjx_sim_info(const mjxSim* s, int32_t* out) {
  if (!s || !out) return fail("null argument");
  const int32_t v[8] = {s->d.nconmax, s->d.njmax, s->big ? s->dbig.nconmax : s->d.nconmax,
                        s->big ? s->dbig.njmax : s->d.njmax, s->spec, s->spec_big, s->ovf_cap,
                        s->nrowclass};
  for (int i = 0; i < 8; i++) out[i] = v[i];
  return 0;
}

int mjx_marker(int tag, void* stream) {
  hipError_t e = mjx::launch_marker(tag, (hipStream_t)stream);
  if (e != hipSuccess) return fail(std::string("marker launch: ") + hipGetErrorString(e));
  return 0;
}

int mjx_sim_stats(mjxSim* s, int32_t* out, void* stream) {
  if (!s || !out) return fail("null argument");
  // per-world counters -> totals: [0] max contacts, [1] max rows, [2..4] overflow /
  // row-overflow / unsupported-pair events, [5] max Newton iterations
  std::vector<int32_t> ws((size_t)s->nworld * 8);
  HIPCHK(hipMemcpyAsync(ws.data(), s->dd.wstats, sizeof(int32_t) * ws.size(), hipMemcpyDeviceToHost,
                        (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  int32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int w = 0; w < s->nworld; w++) {
    const int32_t* x = ws.data() + 8 * (size_t)w;
    r[0] = std::max(r[0], x[0]); r[1] = std::max(r[1], x[1]); r[5] = std::max(r[5], x[5]);
    r[2] += x[2]; r[3] += x[3]; r[4] += x[4];
  }
  // [6] overflow re-solves (worlds re-solved at the max capacity) over all worlds
  HIPCHK(hipMemcpyAsync(&r[6], s->dd.evtotal + 3, sizeof(int32_t), hipMemcpyDeviceToHost,
                        (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  for (int i = 0; i < 8; i++) out[i] = r[i];
  return 0;
}

}  // extern "C"
