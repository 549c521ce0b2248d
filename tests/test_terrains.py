"""Heightfield terrain on CPU: the generator and the oracle's
heightfield narrowphase.

Generator pins (restating `terrains/heightfield_terrains.py` closed forms): grid shapes
(80 x 80 pixels for 8 m at 0.1 m), [0, 1] normalisation, pyramid slope height, wave
amplitude, spawn origins and patch placement (`terrain_generator.py:194-206`), seeded
determinism.  Narrowphase pins: a flat heightfield gives exactly the plane's contacts
(same count, depth, point and normal), and a ramp gives the ramp's normal.
"""

import copy

import numpy as np
import pytest

import oracle_lib as ol
from mjlab_amd import terrains as T
from mjlab_amd.scenes import load_scene


def test_generator_deterministic_and_shapes():
  a_h, a_o = T.TerrainGenerator(T.hf_rough_terrains_cfg(seed=0)).generate()
  b_h, b_o = T.TerrainGenerator(T.hf_rough_terrains_cfg(seed=0)).generate()
  c_h, _ = T.TerrainGenerator(T.hf_rough_terrains_cfg(seed=1)).generate()
  assert len(a_h) == 200 and a_o.shape == (10, 20, 3)
  for x, y in zip(a_h, b_h):
    assert x.pos == y.pos and x.size == y.size and np.array_equal(x.data, y.data)
  assert any(not np.array_equal(x.data, y.data) for x, y in zip(a_h, c_h))
  for h in a_h:
    assert h.data.shape == (80, 80) and h.data.dtype == np.float32
    assert h.data.min() >= 0.0 and h.data.max() <= 1.0
    assert h.size[0] == 4.0 and h.size[1] == 4.0
  np.testing.assert_array_equal(a_o, b_o)


def test_patch_placement_and_origins():
  cfg = T.hf_rough_terrains_cfg(seed=0)
  gen = T.TerrainGenerator(cfg)
  hf, origins = gen.generate()
  # random layout: patch k = (row, col) in row-major order; corner = grid offset + index*size
  for k, h in enumerate(hf):
    r, c = divmod(k, 20)
    corner = np.array([-40.0 + 8.0 * r, -80.0 + 8.0 * c])
    np.testing.assert_allclose(np.array(h.pos[:2]) - corner, [4.0, 4.0])
    np.testing.assert_allclose(origins[r, c, :2], corner + 4.0)


def test_pyramid_and_wave_closed_forms():
  rng = np.random.default_rng(0)
  p = T.HfPyramidSlopedTerrainCfg(slope_range=(0.0, 1.0), platform_width=2.0, border_width=0.25,
                                  size=(8.0, 8.0))
  hf, origin = p.function(0.5, rng)
  # slope 0.5, border 2 px, inner 76 px: height_max = int(0.5 * 7.6 / 2 / 0.005) = 380
  # counts; the platform edge (pixel 38 - 10 = 28) clips at rint(380 (28/38)^2) = 206 counts
  assert hf["size"][2] == pytest.approx(206 * 0.005)
  assert origin[2] == pytest.approx(hf["size"][2])        # spawn on top of the pyramid
  assert hf["pos"][2] == 0.0
  assert hf["data"][0, 0] == 0.0 and hf["data"][40, 40] == pytest.approx(1.0)
  inv = T.HfPyramidSlopedTerrainCfg(slope_range=(0.0, 1.0), platform_width=2.0, border_width=0.25,
                                    inverted=True, size=(8.0, 8.0))
  hfi, oi = inv.function(0.5, rng)
  assert hfi["pos"][2] == pytest.approx(-hfi["size"][2]) and oi[2] == pytest.approx(-hfi["size"][2])
  w = T.HfWaveTerrainCfg(amplitude_range=(0.0, 0.2), num_waves=4, border_width=0.0, size=(8.0, 8.0))
  hw, ow = w.function(1.0, rng)
  # amplitude 0.2 -> 20 counts; cos + sin spans [-2, 2] * 20 (up to rounding)
  assert hw["size"][2] == pytest.approx(80 * 0.005, abs=2 * 0.005)
  assert hw["pos"][2] == pytest.approx(-hw["size"][2] / 2) and ow[2] == 0.0
  assert hw["size"][3] == pytest.approx(0.25 * hw["size"][2])


def test_pairs_put_hfields_last():
  m = load_scene("g1_jump_hfield")
  t = m.geom_type[m.pair_geom1]
  nreg = int(np.argmax(t == 1))
  assert (t[:nreg] != 1).all() and (t[nreg:] == 1).all()
  g1 = m.pair_geom1[nreg:]
  assert (np.diff(g1) >= 0).all()  # grouped by hfield geom
  assert len(np.unique(g1)) == 200


def _flat_hfield_model():
  """The config-5 scene with every heightfield flattened onto z = 0."""
  m = copy.deepcopy(load_scene("g1_jump_hfield"))
  m.arrays["hfield_data"] = np.zeros_like(m.arrays["hfield_data"])
  gp = m.arrays["geom_pos"].copy()
  gp[m.geom_type == 1, 2] = 0.0
  m.arrays["geom_pos"] = gp
  return m


def test_flat_hfield_equals_plane():
  mh, mp = _flat_hfield_model(), load_scene("g1_jump")
  o = mh.arrays["terrain_origins"]
  jq = np.array([mp.jnt_qposadr[j] for j in mp.actuator_trnid])
  for (r, c) in ((3, 5), (7, 12)):
    q = mp.key_qpos.copy()
    q[:2] = o[r, c, :2] + [0.3, -0.2]
    q[2] = 0.55
    fh = ol.forward(mh, q, ctrl=q[jq])
    fp = ol.forward(mp, q, ctrl=q[jq])
    assert fh["ncon"] == fp["ncon"] and fh["ncon"] > 20
    # oracle contact rows: [geom1, geom2, dist, pos(3), normal(3)]; geom ids differ between
    # the two scenes (200 hfields vs 1 plane), so compare the geometry sorted by position
    key = lambda a: np.lexsort((a[:, 5], a[:, 4], a[:, 3]))
    ch, cp = fh["contact"], fp["contact"]
    ch, cp = ch[key(ch)], cp[key(cp)]
    np.testing.assert_allclose(ch[:, 2:9], cp[:, 2:9], atol=1e-9)
    np.testing.assert_allclose(fh["qacc"], fp["qacc"], rtol=1e-6, atol=1e-6)


def test_ramp_normal():
  m = _flat_hfield_model()
  o = m.arrays["terrain_origins"]
  hid = 3 * 20 + 5  # patch (3, 5)
  nr, nc = int(m.hfield_nrow[hid]), int(m.hfield_ncol[hid])
  slope = 0.2  # rise per metre along x (columns span x)
  sx = float(m.hfield_size[hid, 0])
  z = (np.arange(nc) * (2 * sx / (nc - 1))) * slope  # height at column c
  zmax = float(z.max())
  data = m.arrays["hfield_data"].copy()
  adr = int(m.hfield_adr[hid])
  data[adr:adr + nr * nc] = np.tile(z / zmax, nr)
  m.arrays["hfield_data"] = data
  hs = m.arrays["hfield_size"].copy()
  hs[hid, 2] = zmax
  m.arrays["hfield_size"] = hs
  q = m.key_qpos.copy()
  cx, cy = o[3, 5, :2]
  q[:2] = (cx, cy)
  x_local = 0.0  # patch centre: surface height = slope * sx
  q[2] = 0.55 + slope * (x_local + sx) + 0.01
  jq = np.array([m.jnt_qposadr[j] for j in m.actuator_trnid])
  f = ol.forward(m, q, ctrl=q[jq])
  gh = f["contact"][:, 0].astype(int)
  ramp = f["contact"][m.geom_type[gh] == 1]
  assert len(ramp) > 0
  n = np.array([-slope, 0.0, 1.0]) / np.hypot(slope, 1.0)
  for row in ramp:
    np.testing.assert_allclose(row[6:9], n, atol=1e-6)
