"""Per-phase LDS carve sizes and resident worlds per CU (host replica of make_lds in
csrc/engine.hip; diagnostic only -- keep in step with the Spec table there)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
from mjlab_amd.scenes import load_scene


def carve(m, ph, C, R):
  nb, nv = m.nbody, (m.nv + 3) & ~3
  A, B, Cp = 1, 2, 4
  spec = [("ints", 8, A | B | Cp), ("qpos", m.nq, A | Cp), ("qvel", nv, A | Cp), ("ctrl", m.nu, A),
          ("qacc_ws", nv, B | Cp), ("qfrc_applied", nv, A), ("xfrc", 6 * nb, 0),
          ("xpos", 3 * nb, A), ("xquat", 4 * nb, A), ("xmat", 9 * nb, A), ("xipos", 3 * nb, A),
          ("ximat", 9 * nb, A), ("xanchor", 3 * m.njnt, A), ("xaxis", 3 * m.njnt, A),
          ("stmass", nb, A), ("subtree_com", 3 * nb, A | Cp), ("cinert", 10 * nb, A),
          ("crb", 10 * nb, A), ("cvel", 6 * nb, A | Cp), ("cacc", 6 * nb, A | Cp),
          ("stlin", 3 * nb, A), ("stang", 3 * nb, A), ("cdof", 6 * nv, A | Cp),
          ("cdofdot", 6 * nv, A | Cp), ("gxpos", 3 * int((m.geom_type != 1).sum()), A),
          ("gxmat", 9 * int((m.geom_type != 1).sum()), A),
          ("sxpos", 3 * m.nsite, A | Cp), ("sxmat", 9 * m.nsite, A | Cp), ("M", nv * nv, A | B),
          ("H", nv * nv, A | B), ("qfrc_bias", nv, A), ("qfrc_passive", nv, A),
          ("qfrc_act", nv, A), ("qfrc_smooth", nv, A | B | Cp), ("qacc_smooth", nv, A | B),
          ("x", nv, B | Cp), ("Mx", nv, B), ("grad", nv, 0), ("srch", nv, B), ("Ms", nv, B),
          ("qfrc_con", nv, B | Cp), ("vtmp", nv, 0), ("act_force", m.nu, A | Cp),
          ("act_len", m.nu, A), ("act_vel", m.nu, A), ("con_g1", C, A | Cp), ("con_g2", C, A | Cp),
          ("con_key", C, A), ("con_dist", C, A | Cp), ("con_pos", 3 * C, A | Cp),
          ("con_frame", 9 * C, A | Cp), ("con_mu", 2 * C, A | Cp), ("con_kb", 2 * C, A),
          ("con_imp", C, A), ("con_imargin", C, A), ("con_dim", C, A | Cp),
          ("con_efc", C, A | Cp), ("efc_J", R * nv, B), ("efc_aref", R, A | B), ("efc_D", R, A | B),
          ("efc_jar", R, B), ("efc_Js", R, B), ("efc_force", R, B | Cp), ("efc_cid", R, A),
          ("efc_act", R, B), ("hdiag", nv, 0), ("red", 5 * 64, B)]
  n = {k: v for k, v, _ in spec}
  L, o = {}, 0

  def take(f):
    nonlocal o
    if f in L: return
    L[f] = o
    o += (n[f] + 3) & ~3
  packB = ["ints", "M", "qacc_smooth", "qfrc_smooth", "efc_aref", "efc_D", "efc_J"]
  packC = ["cdof", "cdofdot", "cvel", "subtree_com", "sxpos", "sxmat", "act_force", "con_g1",
           "con_g2", "con_dist", "con_pos", "con_frame", "con_mu", "con_dim", "con_efc",
           "qfrc_smooth", "ints", "x", "qfrc_con", "efc_force"]
  if ph == 1:
    for f in packB: take(f)
    L["H"] = L["red"] = L["M"]; L["efc_Js"] = L["efc_aref"]
  if ph == 2:
    for f in packC: take(f)
  if ph == 0:
    s0 = o
    for f in ["con_g1", "con_g2", "con_key", "con_dist", "con_pos", "con_frame", "con_mu",
              "con_kb", "con_imp", "con_imargin", "con_dim", "con_efc", "efc_aref",
              "efc_D", "efc_cid"]: take(f)
    if o - s0 >= nv * nv: L["M"] = L["H"] = s0
    s1 = o
    for f in ["cinert", "crb", "cacc", "xanchor", "xaxis"]: take(f)
    ngl = int((m.geom_type != 1).sum())
    gp = (3 * ngl + 3) & ~3
    if o - s1 >= gp + 9 * ngl: L["gxpos"] = s1; L["gxmat"] = s1 + gp
  for f, _, mask in spec:
    if mask & (1 << ph): take(f)
  return 4 * o


if __name__ == "__main__":
  for scene, C, R in [("g1_velocity", 48, 160), ("go1_velocity", 48, 160), ("g1_jump_hfield", 48, 160)]:
    m = load_scene(scene)
    out = []
    for ph in range(3):
      b = carve(m, ph, C, R)
      out.append(f"{'ABC'[ph]} {b / 1024:.1f} KB ({160 * 1024 // b}/CU)")
    print(scene, f"nconmax={C} njmax={R}:", ", ".join(out))
