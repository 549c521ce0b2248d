// carve.h — per-phase LDS carves of the step kernels (offsets in 4-byte words).
//
// constexpr so that the model-specialised kernels (specs.inc) get every LDS offset as a
// compile-time immediate; the generic kernels and the host use the same function at run
// time.  Included by engine.h after the Dims / Lds definitions.
#pragma once

#include <initializer_list>
#include <utility>

#ifndef MJX_JTDJ_MFMA
#define MJX_JTDJ_MFMA 0
#endif

namespace mjx {

// register-row length of the dense SPD kernels: exact fits for the shipped robots (Go1 nvp
// 20, G1 nvp 36), multiples of 8 otherwise (engine.hip generic_fn)
constexpr int nr_for_nv(int nv) {
  const int nvp = (nv + 3) & ~3;
  return nvp <= 8 ? 8 : nvp <= 16 ? 16 : nvp <= 20 ? 20 : nvp <= 24 ? 24 : nvp <= 32 ? 32
       : nvp <= 36 ? 36 : nvp <= 40 ? 40 : nvp <= 48 ? 48 : nvp <= 56 ? 56 : 64;
}

// Lower-tile rows ("LTR"): the lower triangle of an nvp x nvp matrix (nvp a multiple of 4)
// stored row by row, row i = 4b + r holding its columns [0, 4(b + 1)) -- the 4x4 tiles on and
// left of the diagonal -- at offset 8 b (b + 1) + 4 (b + 1) r.  Dense (chunk k of 4 floats is
// at 4k), 16-byte aligned rows, 8 nb (nb + 1) floats in all (720 for nvp 36 instead of 1296).
// The phase hand-offs of the symmetric M (A -> B) and of the implicit-integration factor
// (A -> C) use it, and phase B stages the Newton Hessian and its factor in it.
constexpr int ltr_off(int i) { return 8 * (i >> 2) * ((i >> 2) + 1) + 4 * ((i >> 2) + 1) * (i & 3); }
constexpr int ltr_size(int nvp) { return 8 * (nvp >> 2) * ((nvp >> 2) + 1); }

// Phase carves.  Masks: A = 1 (kinematics .. constraint rows), B = 2 (Newton), C = 4
// (post/integrate).  A phase carve holds only the regions that phase touches (the rest sit
// past the allocation and are never accessed).  Phase inputs are carved FIRST, in a fixed
// order, so the per-world global scratch holds them as one contiguous "pack" with the same
// internal offsets: B pack = [ints M qacc_smooth qfrc_smooth efc_aref efc_D efc_J] (J last,
// so only the live rows are copied; M's slot holds M in LTR form, the rest of the slot is
// neither written nor read), C pack = [A outputs | B outputs].  Each phase then fills its
// inputs with one or two bulk copies.
// jglobal (phase B only): the Newton reads the constraint Jacobian straight from the B pack in
// global memory (L2) instead of an LDS copy -- the carve of the latency Newton kernel's heavy
// worlds, whose J (up to njmax x nvp floats) is most of the full-capacity carve
constexpr Lds make_lds(const Dims& d, int ph, bool jglobal = false) {
  Lds L{};
  const int nb = d.nbody, nv = (d.nv + 3) & ~3, C = d.nconmax, R = d.njmax;  // nv padded
  constexpr int A = 1, B = 2, Cp = 4;
  // M's slot: phase A factors M in full form; phase B holds M in LTR form and stages the
  // Newton Hessian and its factor in the same form (the MFMA J^T D J variant keeps the full
  // one), and the slot also takes jt_mul's partial sums (red)
  const int mslot = ph == 1 && !MJX_JTDJ_MFMA
                        ? (ltr_size(nv) > 5 * kWave ? ltr_size(nv) : 5 * kWave) : nv * nv;
  struct Slot { int Lds::*f; int n; int mask; };
  const Slot all[] = {
    {&Lds::ints, 8, A | B | Cp},
    // ctrl, qfrc_applied, subtree masses, qfrc_bias / passive and actuator length / velocity
    // live in lane registers in phase A; body rotations as quaternions (xmat / ximat are
    // formed where used)
    {&Lds::qpos, d.nq, A | Cp}, {&Lds::qvel, nv, A | Cp}, {&Lds::ctrl, d.nu, 0},
    {&Lds::qacc_ws, nv, B | Cp}, {&Lds::qfrc_applied, nv, 0}, {&Lds::xfrc, 6 * nb, 0},  // xfrc read from HBM (rare)
    {&Lds::xpos, 3 * nb, A}, {&Lds::xquat, 4 * nb, A}, {&Lds::xmat, 9 * nb, 0},
    {&Lds::xipos, 3 * nb, A}, {&Lds::ximat, 9 * nb, 0}, {&Lds::xanchor, 3 * d.njnt, A},
    {&Lds::xaxis, 3 * d.njnt, A}, {&Lds::stmass, nb, 0}, {&Lds::subtree_com, 3 * nb, A | Cp},
    {&Lds::cinert, 10 * nb, A}, {&Lds::crb, 10 * nb, A}, {&Lds::cvel, 6 * nb, A | Cp},
    {&Lds::cacc, 6 * nb, A | Cp}, {&Lds::stlin, 3 * nb, A}, {&Lds::stang, 3 * nb, A},
    // cdofdot: phase A only, in the crb slot (below); phase C gets the velocity-product
    // acceleration cacc_v(b) = -gravity + sum cdofdot * qvel (6 per body) that A's RNE forms
    {&Lds::cdof, 6 * nv, A | Cp}, {&Lds::cdofdot, 6 * nv, 0}, {&Lds::cacc_v, 6 * nb, Cp},
    {&Lds::gxpos, 3 * d.ngeom_lds, A}, {&Lds::gxmat, 9 * d.ngeom_lds, A},
    {&Lds::sxpos, 3 * d.nsite, A | Cp}, {&Lds::sxmat, 9 * d.nsite, A | Cp},
    {&Lds::M, mslot, A | B}, {&Lds::H, nv * nv, A | B},
    // phase A keeps qfrc_actuator / qfrc_smooth in lane registers and the smooth solve's
    // qacc_smooth in dead cinert space (below)
    {&Lds::qfrc_bias, nv, 0}, {&Lds::qfrc_passive, nv, 0}, {&Lds::qfrc_act, nv, 0},
    {&Lds::qfrc_smooth, nv, B | Cp}, {&Lds::qacc_smooth, nv, B}, {&Lds::x, nv, B | Cp},
    {&Lds::Mx, nv, B}, {&Lds::grad, nv, 0}, {&Lds::srch, nv, B}, {&Lds::Ms, nv, B},
    {&Lds::qfrc_con, nv, B | Cp}, {&Lds::vtmp, nv, 0},
    {&Lds::act_force, d.nu, 0}, {&Lds::act_len, d.nu, 0}, {&Lds::act_vel, d.nu, 0},
    {&Lds::con_g1, C, A | Cp}, {&Lds::con_g2, C, A | Cp}, {&Lds::con_key, C, A},
    {&Lds::con_dist, C, A | Cp}, {&Lds::con_pos, 3 * C, A | Cp}, {&Lds::con_frame, 9 * C, 0},
    {&Lds::con_n, 3 * C, A | Cp},  // unit normals: cframe() rebuilds the frame where used
    {&Lds::con_mu, 2 * C, A | Cp}, {&Lds::con_kb, 2 * C, A}, {&Lds::con_imp, C, A},
    {&Lds::con_imargin, C, A}, {&Lds::con_dim, C, A | Cp}, {&Lds::con_efc, C, A | Cp},
    {&Lds::efc_J, ph == 1 && jglobal ? 0 : R * nv, B},  // phase A writes J rows straight into the B pack
    {&Lds::efc_aref, R, A | B}, {&Lds::efc_D, R, A | B}, {&Lds::efc_jar, R, B},
    {&Lds::efc_Js, R, B}, {&Lds::efc_force, R, B | Cp}, {&Lds::efc_cid, R > nb ? R : nb, A},
    {&Lds::efc_act, R, B}, {&Lds::hdiag, nv, 0},
    {&Lds::red, 5 * kWave, B},
    // column-block broadcast buffer of the blocked Cholesky (rows_chol): 4 floats per lane;
    // aliased below into a region that is dead while a factorization runs
    {&Lds::chol, 4 * kWave, 0},
  };
  int Lds::* const packB[] = {&Lds::ints, &Lds::M, &Lds::qacc_smooth, &Lds::qfrc_smooth,
                                     &Lds::efc_aref, &Lds::efc_D, &Lds::efc_J};
  // C pack: first what every substep reads (the contact air times' geom matches, the
  // integration's smooth force), then what only the last substep of a fused step reads (the
  // acc-stage sensors, contact forces and outputs), then phase B's part
  int Lds::* const packC[] = {
      &Lds::con_g1, &Lds::con_g2, &Lds::qfrc_smooth,
      &Lds::cdof, &Lds::cacc_v, &Lds::cvel, &Lds::subtree_com, &Lds::sxpos, &Lds::sxmat,
      &Lds::con_dist, &Lds::con_pos, &Lds::con_n, &Lds::con_mu, &Lds::con_dim, &Lds::con_efc,
      // written by phase B:
      &Lds::ints, &Lds::x, &Lds::qfrc_con, &Lds::efc_force};
  constexpr int kAbsent = 1 << 24;
  for (const Slot& sp : all) L.*(sp.f) = kAbsent;
  int o = 0;
  auto take = [&](int Lds::*f) {
    if (L.*f != kAbsent) return;
    for (const Slot& sp : all)
      if (sp.f == f) { L.*f = o; o += (sp.n + 3) & ~3; return; }  // 16-B aligned carve
  };
  if (ph == 1) for (auto f : packB) take(f);
  if (ph == 2) {
    for (auto f : packC) {
      take(f);
      if (f == &Lds::qfrc_smooth) L.packC_sub = o;
    }
  }
  L.pack_len = o;
  L.packC_b = ph == 2 ? L.ints : 0;  // start of the phase-B-written part of the C pack
  if (ph == 1) {
    // Phase B holds M in register tiles for the whole solve (tiles_symv), so M's pack slot
    // is reused as the Cholesky staging area H and as jt_mul's partial sums; the line-search
    // direction J s reuses efc_aref (only read by the warmstart).
    L.H = L.M;
    L.red = L.M;
    L.efc_Js = L.efc_aref;
    // the Cholesky stages H in M's slot: rows are loaded before the first column block is
    // published and the factor is stored after the last (LDS ops of a wave run in order)
    if (mslot >= 4 * kWave) L.chol = L.M;
  }
  if (ph == 0) {
    // Phase A stage order is kinematics, com, CRB/M, RNE, smooth solve, subtree momenta,
    // collision, contacts, rows.  The aliases follow from it:
    //  - joint anchors / axes (dead after cdof), then M and H (the smooth solve's in-place
    //    factor) live in the contact/row block, which is first written by collision, after
    //    the smooth solve;
    //  - the subtree momenta (written after RNE, read back before the geom frames), then
    //    the geom frames (computed at the start of collision) live in [cinert crb cacc],
    //    dead once RNE has run.
    auto group = [&](std::initializer_list<int Lds::*> fs) {
      const int start = o;
      for (auto f : fs) take(f);
      return std::make_pair(start, o - start);
    };
    auto g1 = group({&Lds::con_g1, &Lds::con_g2, &Lds::con_key, &Lds::con_dist, &Lds::con_pos,
                     &Lds::con_n, &Lds::con_mu, &Lds::con_kb, &Lds::con_imp,
                     &Lds::con_imargin, &Lds::con_dim, &Lds::con_efc, &Lds::efc_aref, &Lds::efc_D,
                     &Lds::efc_cid});
    // M (assembled after CRB, copied to the B/C packs at once, factored in place by the
    // smooth solve) is dead before collision: M and H share the contact/row block too.
    if (g1.second >= nv * nv) L.M = L.H = g1.first;
    // joint anchors / axes: from kinematics to cdof, before M is assembled; the kinematics
    // ancestor-pointer scratch sits in efc_cid, past them
    const int nj3 = (3 * d.njnt + 3) & ~3;
    if (g1.second >= 2 * nj3 && L.efc_cid >= g1.first + 2 * nj3) {
      L.xanchor = g1.first;
      L.xaxis = g1.first + nj3;
    }
    auto g2 = group({&Lds::cinert, &Lds::crb, &Lds::cacc});
    // subtree momenta in the cinert slot (crb holds their mass scratch)
    const int nb3 = (3 * nb + 3) & ~3;
    if (10 * nb >= 2 * nb3) {
      L.stlin = L.cinert;
      L.stang = L.cinert + nb3;
    }
    // cdofdot lives from comVel to RNE's acceleration sum, in the crb slot: M is assembled
    // (crb dead) and RNE's body forces are written there only after that sum
    if (10 * nb >= 6 * nv) L.cdofdot = L.crb;
    else take(&Lds::cdofdot);
    // qacc_smooth (the smooth solve's right-hand side, then its solution; phase A stores it
    // to the B pack right after the solve) in cinert's tail past the subtree momenta:
    // cinert is dead after RNE, and the geom frames land there only at collision
    int mom_end = L.stlin == L.cinert ? g2.first + 2 * nb3 : g2.first;
    if (L.stlin == L.cinert && 10 * nb >= 2 * nb3 + nv) {
      L.qacc_smooth = mom_end;
      mom_end += nv;
    } else {
      take(&Lds::qacc_smooth);
    }
    const int gp = (3 * d.ngeom_lds + 3) & ~3;
    if (g2.second >= gp + 9 * d.ngeom_lds) {
      L.gxpos = g2.first;
      L.gxmat = g2.first + gp;
    }
    // both phase-A factorizations (implicit-integration factor, smooth solve) run after RNE
    // and before the geom frames are computed: the same dead group holds the Cholesky buffer,
    // at its tail (the subtree momenta at its head are live across the factorizations)
    if (g2.first + g2.second - 4 * kWave >= mom_end) L.chol = g2.first + g2.second - 4 * kWave;
  }
  const int bit = 1 << ph;
  for (const Slot& sp : all)
    if (sp.mask & bit) take(sp.f);
  if (ph <= 1) take(&Lds::chol);  // no alias fitted: a slot of its own
  L.total = o;
  return L;
}

}  // namespace mjx
