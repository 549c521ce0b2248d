"""Box-stair rough terrain on CPU: the generator, the compiled scene's
terrain pair tail, the terrain-level curriculum update, and the oracle's box narrowphase.

Generator pins (restating `terrains/primitive_terrains.py` / `terrains/utils.py` closed
forms): pyramid / inverted-pyramid stairs tile the patch with one box per point, every step
top at its step height, the spawn origin on the platform; ROUGH_TERRAINS_CFG's curriculum
layout (`terrain_generator.py:149-175`) and the grid border.  Narrowphase pins: a flat box
patch gives the plane's contacts (same depth and point, opposite normal: the robot geom is
geom 1 against a box), a capsule crossing a box edge touches at the edge, a sphere centre
inside a box leaves through the nearest face.  The box narrowphase restates MuJoCo's
sphere-box semantics; capsule-box is this build's segment search (parity with mujoco_warp's
capsule_box unpinned).
"""

import copy

import numpy as np
import pytest
import torch

import oracle_lib as ol
from mjlab_amd import terrains as T
from mjlab_amd.compiler.mjcf import parse_mjcf_string
from mjlab_amd.compiler.model import BoxSpec, EntitySpec, compile_scene
from mjlab_amd.scenes import load_scene


def _top_at(boxes, x, y):
  """Highest box top over (x, y) and how many boxes contain the point."""
  tops = [p[2] + s[2] for p, s in boxes
          if abs(x - p[0]) < s[0] and abs(y - p[1]) < s[1]]
  return (max(tops) if tops else None), len(tops)


@pytest.mark.parametrize("inverted", [False, True])
def test_stairs_tile_the_patch_with_step_heights(inverted):
  cls = T.BoxInvertedPyramidStairsTerrainCfg if inverted else T.BoxPyramidStairsTerrainCfg
  c = cls(step_height_range=(0.0, 0.1), step_width=0.3, platform_width=3.0, border_width=1.0,
          size=(8.0, 8.0))
  boxes, origin = c.function(0.5, None)
  h = 0.05
  # (8 - 2 - 3) // 0.6 + 1 = 6 steps: 4 boxes each, the platform, 4 border boxes
  assert len(boxes) == 6 * 4 + 1 + 4
  assert origin[:2].tolist() == [4.0, 4.0]
  assert origin[2] == pytest.approx(-7 * h if inverted else 7 * h)
  rng = np.random.default_rng(0)
  for x, y in rng.uniform(1.0 + 1e-3, 7.0 - 1e-3, (400, 2)):
    ring = int((3.0 - max(abs(x - 4.0), abs(y - 4.0))) // 0.3)  # 0 = outermost step
    if ring < 0 or abs(max(abs(x - 4.0), abs(y - 4.0)) - (3.0 - 0.3 * (ring + 1))) < 1e-6:
      continue
    top, cnt = _top_at(boxes[4:], x, y)
    assert cnt == 1  # one box under every point of the stairs (no overlaps, no gaps)
    k = min(ring, 6)
    want = -(k + 1) * h if inverted else (k + 1) * h
    assert top == pytest.approx(want)
  # the border ring sits on the outer metre, its top at z = 0
  top, cnt = _top_at(boxes[:4], 0.5, 4.0)
  assert cnt == 1 and top == pytest.approx(0.0)


def test_rough_curriculum_layout_and_border():
  cfg = T.rough_terrains_cfg(seed=0, curriculum=True)
  gen = T.TerrainGenerator(cfg)
  geoms, origins = gen.generate()
  assert origins.shape == (10, 20, 3)
  assert all(isinstance(g, BoxSpec) for g in geoms)
  assert [g.name for g in geoms] == [f"terrain_{k}" for k in range(len(geoms))]
  # proportions 0.4 / 0.3 / 0.3 over 20 columns: 8 flat, 6 stairs, 6 inverted stairs
  assert len(geoms) == 8 * 10 * 1 + 12 * 10 * 29 + 4
  # curriculum: column-major, difficulty (row + U) / 10 -> platform height grows with the row
  for col, sign in ((9, 1.0), (16, -1.0)):
    z = origins[:, col, 2] * sign
    assert (np.diff(z) > 0).all()
    assert (z >= 0).all() and (z < 7 * 0.1 + 1e-9).all()
    for row in range(10):
      assert row * 0.07 - 1e-9 <= z[row] <= (row + 1) * 0.07 + 1e-9  # 7 h, h = 0.1 d
  np.testing.assert_allclose(origins[:, :8, 2], 0.0)
  # the grid border: 4 boxes of 20 m around the 80 m x 160 m grid, tops at z = 0
  border = geoms[-4:]
  for b in border:
    assert b.pos[2] + b.size[2] == pytest.approx(0.0)
  assert border[0].pos[1] - border[0].size[1] == pytest.approx(80.0)
  assert border[2].pos[0] + border[2].size[0] == pytest.approx(-40.0)


def test_rough_scene_terrain_pair_tail():
  m = load_scene("g1_velocity_rough")
  gt, body = m.geom_type, m.geom_bodyid
  static = (gt == 6) & (m.body_weldid[body] == 0)
  assert static.sum() == 3564 and (gt[static] == 6).all()
  p1, p2 = m.pair_geom1, m.pair_geom2
  tail = static[p1] | static[p2]
  nreg = int(np.argmax(tail))
  assert not tail[:nreg].any() and tail[nreg:].all()
  assert nreg == load_scene("g1_velocity").npair - 33  # the plane's 33 pairs move to the boxes
  sg = p2[nreg:]  # the box is geom 2 (higher geom type) of every terrain pair
  assert static[sg].all() and not static[p1[nreg:]].any()
  assert (np.diff(sg) >= 0).all()
  _, counts = np.unique(sg, return_counts=True)
  assert (counts == 33).all()  # every robot geom that met the plane meets every box
  np.testing.assert_allclose(m.arrays["terrain_size"], [8.0, 8.0])
  assert m.arrays["sensor_geommask1"].shape[1] == (m.ngeom + 31) // 32


def test_masked_terrain_update_matches_reference_rule():
  from mjlab_amd.scene import Terrain
  o = np.zeros((10, 4, 3))
  o[..., 0] = np.arange(10)[:, None]
  o[..., 1] = np.arange(4)[None, :]
  torch.manual_seed(0)
  a = Terrain(o, (8.0, 8.0), 64, "cpu", max_init_terrain_level=5)
  b = copy.deepcopy(a)
  assert int(a.terrain_levels.max()) <= 5
  g = torch.Generator().manual_seed(1)
  for _ in range(20):
    mask = torch.rand(64, generator=g) < 0.3
    up = torch.rand(64, generator=g) < 0.4
    down = (torch.rand(64, generator=g) < 0.4) & ~up
    ids = mask.nonzero().squeeze(-1)
    # past the top level an env wraps to a random level: the two forms draw differently
    wrap = mask & (a.terrain_levels + up.long() - down.long() >= 10)
    a.update_env_origins(ids, up[ids], down[ids])
    b.update_env_origins_masked(mask, up, down)
    assert torch.equal(a.terrain_levels[~wrap], b.terrain_levels[~wrap])
    assert (b.terrain_levels[wrap] < 10).all()
    b.terrain_levels[wrap] = a.terrain_levels[wrap]
    b.env_origins.copy_(b.terrain_origins[b.terrain_levels, b.terrain_types])
  torch.testing.assert_close(a.env_origins, b.env_origins)
  assert float(b.mean_level) == pytest.approx(float(b.terrain_levels.float().mean()))
  np.testing.assert_array_equal(a.terrain_types.numpy(), np.arange(64) // 16)


def test_flat_box_patch_equals_plane():
  mr, mp = load_scene("g1_velocity_rough"), load_scene("g1_velocity")
  o = mr.arrays["terrain_origins"]
  jq = np.array([mp.jnt_qposadr[j] for j in mp.actuator_trnid])
  for (r, c) in ((3, 2), (8, 6)):
    q = mp.key_qpos.copy()
    q[:2] = o[r, c, :2] + [0.4, -0.7]
    q[2] = 0.74
    q[7:] += np.random.default_rng(r).uniform(-0.05, 0.05, mp.nq - 7)
    fr = ol.forward(mr, q, ctrl=q[jq])
    fp = ol.forward(mp, q, ctrl=q[jq])
    assert fr["ncon"] == fp["ncon"] and fr["ncon"] >= 4
    key = lambda a: np.lexsort((a[:, 5], a[:, 4], a[:, 3]))
    cr, cp = fr["contact"], fp["contact"]
    cr, cp = cr[key(cr)], cp[key(cp)]
    np.testing.assert_allclose(cr[:, 2:6], cp[:, 2:6], atol=1e-9)   # depth, point
    np.testing.assert_allclose(cr[:, 6:9], -cp[:, 6:9], atol=1e-12)  # normal reversed
    np.testing.assert_allclose(fr["qacc"], fp["qacc"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(fr["sensordata"], fp["sensordata"], rtol=1e-6, atol=1e-6)


_CAPSULE = """<mujoco><worldbody>
  <body name="cap" pos="0 0 1"><freejoint/>
    <inertial pos="0 0 0" mass="1" diaginertia="0.01 0.01 0.01"/>
    <geom name="c" type="{type}" size="{size}"/></body>
</worldbody></mujoco>"""


def _probe(gtype, size):
  xml = parse_mjcf_string(_CAPSULE.format(type=gtype, size=size))
  ent = EntitySpec("probe", xml)
  box = BoxSpec("terrain_0", pos=(0.0, 0.0, -0.5), size=(1.0, 1.0, 0.5))  # top z = 0, x in [-1, 1]
  return compile_scene([ent], terrain="generator", terrain_geoms=[box], timestep=0.005)


def _quat_y(angle):
  return np.array([np.cos(angle / 2), 0.0, np.sin(angle / 2), 0.0])


def test_capsule_across_a_box_edge_touches_at_the_edge():
  m = _probe("capsule", "0.05 0.2")
  th = 0.3  # axis (local z) turned onto +x and tipped down by th: the +x end is lower
  q = np.zeros(7)
  q[:3] = (1.0, 0.0, 0.04)
  q[3:] = _quat_y(np.pi / 2 + th)
  f = ol.forward(m, q)
  assert f["ncon"] == 1  # the ends are clear (one above the top, one past the side)
  c = f["contact"][0]
  # closest segment point: the foot of the perpendicular from the edge (1, 0, 0) onto the
  # axis, at t = 0.04 sin(th) past the centre, 0.04 cos(th) from the edge
  s, co = np.sin(th), np.cos(th)
  p = np.array([1.0 + 0.04 * s * co, 0.0, 0.04 - 0.04 * s * s])
  n = np.array([-s, 0.0, -co])
  assert c[2] == pytest.approx(0.04 * co - 0.05, abs=1e-6)
  np.testing.assert_allclose(c[6:9], n, atol=1e-5)
  np.testing.assert_allclose(c[3:6], 0.5 * (np.array([1.0, 0, 0]) + p + n * 0.05), atol=1e-6)
  # lying flat on the top face: the two ends, as plane-capsule
  q[:3] = (0.0, 0.3, 0.045)
  q[3:] = _quat_y(np.pi / 2)
  f = ol.forward(m, q)
  assert f["ncon"] == 2
  np.testing.assert_allclose(f["contact"][:, 2], [-0.005, -0.005], atol=1e-9)
  np.testing.assert_allclose(np.sort(f["contact"][:, 3]), [-0.2, 0.2], atol=1e-9)


def test_sphere_centre_inside_a_box_leaves_through_the_nearest_face():
  m = _probe("sphere", "0.05")
  q = np.zeros(7)
  q[:3] = (0.98, 0.0, -0.3)
  q[3] = 1.0
  f = ol.forward(m, q)
  assert f["ncon"] == 1
  c = f["contact"][0]
  assert c[2] == pytest.approx(-0.02 - 0.05)
  np.testing.assert_allclose(c[6:9], [-1.0, 0.0, 0.0], atol=1e-12)
  np.testing.assert_allclose(c[3:6], [0.98 - 0.015, 0.0, -0.3], atol=1e-12)


def _quat_mul(a, b):
  return np.array([a[0]*b[0]-a[1]*b[1]-a[2]*b[2]-a[3]*b[3], a[0]*b[1]+a[1]*b[0]+a[2]*b[3]-a[3]*b[2],
                   a[0]*b[2]-a[1]*b[3]+a[2]*b[0]+a[3]*b[1], a[0]*b[3]+a[1]*b[2]-a[2]*b[1]+a[3]*b[0]])


def test_box_resting_on_a_box_face():
  m = _probe("box", "0.2 0.1 0.05")
  q = np.zeros(7)
  q[:3] = (0.3, -0.2, 0.05 - 0.004)  # 4 mm into the top face
  q[3] = 1.0
  f = ol.forward(m, q)
  assert f["ncon"] == 4  # the bottom face's corners
  c = f["contact"]
  assert (c[:, 0] == 0).all() and (c[:, 1] == 1).all()  # static box is geom 1 (index order)
  np.testing.assert_allclose(c[:, 2], -0.004, atol=1e-12)
  np.testing.assert_allclose(c[:, 6:9], np.tile([0.0, 0.0, 1.0], (4, 1)), atol=1e-12)
  np.testing.assert_allclose(np.sort(c[:, 3]), [0.1, 0.1, 0.5, 0.5], atol=1e-12)
  np.testing.assert_allclose(c[:, 5], -0.002, atol=1e-12)  # halfway between the surfaces
  # hanging half over the +x edge: the clip keeps the part over the face
  q[0] = 1.0
  f = ol.forward(m, q)
  assert f["ncon"] == 4
  np.testing.assert_allclose(np.sort(f["contact"][:, 3]), [0.8, 0.8, 1.0, 1.0], atol=1e-12)


def test_box_edge_across_a_box_edge():
  m = _probe("box", "0.2 0.05 0.05")
  # long axis x tipped down toward +x by 0.3 rad, rolled 45 deg about it: its lowest edge
  # (along x) passes beyond the static box's top edge at x = 1 (which runs along y)
  qr = _quat_mul(_quat_y(0.3), np.array([np.cos(np.pi / 8), np.sin(np.pi / 8), 0.0, 0.0]))
  q = np.zeros(7)
  q[:3] = (1.0, 0.1, 0.05 * np.sqrt(2) - 0.01)
  q[3:] = qr
  f = ol.forward(m, q)
  assert f["ncon"] == 1
  c = f["contact"][0]
  assert c[2] < 0.0
  np.testing.assert_allclose(c[3:6], [1.0, 0.1, 0.0], atol=0.02)  # at the static edge
  ex = np.array([np.cos(0.3), 0.0, -np.sin(0.3)])                 # moving edge direction
  n = c[6:9]
  assert abs(n[1]) < 1e-9 and abs(n @ ex) < 1e-9 and n[2] > 0.5   # normal to both edges


def _exact_capsule_box(c, a, hl, s):
  """min over the segment c + t a (|t| <= hl) of the box signed distance (box frame, half
  sizes s), fp64: dense samples, then golden refinement in the best bracket; returns
  (distance, t) -- an oracle-independent restatement of what MuJoCo's first capsule-box
  contact reports (the sphere at the segment point closest to the box)."""
  def sd(t):
    q = c[None, :] + np.atleast_1d(t)[:, None] * a[None, :]
    d = np.abs(q) - s
    out = np.linalg.norm(np.maximum(d, 0.0), axis=1) + np.minimum(d.max(axis=1), 0.0)
    return out
  ts = np.linspace(-hl, hl, 4001)
  v = sd(ts)
  k = int(np.argmin(v))
  lo, hi = ts[max(k - 1, 0)], ts[min(k + 1, len(ts) - 1)]
  for _ in range(80):
    m1, m2 = lo + (hi - lo) * 0.382, lo + (hi - lo) * 0.618
    if sd(m1)[0] <= sd(m2)[0]:
      hi = m2
    else:
      lo = m1
  t = 0.5 * (lo + hi)
  cand = [(float(sd(t)[0]), t), (float(v[k]), ts[k])]
  return min(cand)


def test_capsule_box_deepest_contact_is_the_exact_distance():
  """Against random capsule poses over the box's top face, its +x edge and its corner (the
  stair geometry: axis-aligned boxes under foot capsules), the deepest contact's depth is
  the exact capsule-box distance minus the radius, to 1e-4 (this build's tie band: an
  interior segment point is used when it is deeper than both ends by 1e-4) and to 1e-8
  where the interior point is clearly deeper and outside the box (1e-5 inside it: the
  sphere-box face tie band); contacts <= 2, normals unit."""
  r, hl = 0.05, 0.2
  m = _probe("capsule", f"{r} {hl}")
  s = np.array([1.0, 1.0, 0.5])
  rng = np.random.default_rng(7)
  clear, n_tested = 0, 0
  for i in range(300):
    site = i % 3
    p = np.array([rng.uniform(-0.8, 0.8), rng.uniform(-0.8, 0.8), 0.0])
    if site == 1:
      p[0] = 1.0 + rng.uniform(-0.15, 0.15)
    elif site == 2:
      p[:2] = 1.0 + rng.uniform(-0.15, 0.15, 2)
    p[2] = rng.uniform(-0.02, 0.2)
    u = rng.normal(size=4)
    u /= np.linalg.norm(u)
    q = np.concatenate([p, u])
    f = ol.forward(m, q)
    # capsule axis (local z) in the box frame: the box sits at (0, 0, -0.5), unrotated
    w, x, y, z = u
    a = np.array([2 * (x * z + w * y), 2 * (y * z - w * x), 1 - 2 * (x * x + y * y)])
    c = p - np.array([0.0, 0.0, -0.5])
    dmin, tmin = _exact_capsule_box(c, a, hl, s)
    ends = min(_exact_capsule_box(c + a * hl, a, 0.0, s)[0], _exact_capsule_box(c - a * hl, a, 0.0, s)[0])
    if dmin - r > 0.0:  # separated (margin 0): no contact
      assert f["ncon"] == 0
      continue
    n_tested += 1
    assert 1 <= f["ncon"] <= 2
    con = f["contact"]
    np.testing.assert_allclose(np.linalg.norm(con[:, 6:9], axis=1), 1.0, atol=1e-12)
    deepest = con[:, 2].min()
    # never deeper than the exact distance, but for the inside case's face tie band (a segment
    # point inside the box leaves through the +z face when that is within 1e-5 of the least
    # penetration, so fp32 and fp64 pick the same face)
    assert deepest >= dmin - r - 1e-5 - 1e-9
    if ends - dmin > 2e-4:                     # an interior point is clearly the closest
      clear += 1
      assert deepest == pytest.approx(dmin - r, abs=1e-5 if dmin < 0 else 1e-8)
    else:
      assert deepest <= dmin - r + 1e-4
  assert n_tested > 100 and clear > 10
