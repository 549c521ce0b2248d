"""Procedural terrains (row a30, config 5; row f3, box-stair rough terrain).

Restates the reference's terrain generators:
  * heightfield sub-terrains, `src/mjlab/terrains/heightfield_terrains.py:104-499`
    (HfPyramidSlopedTerrainCfg, HfRandomUniformTerrainCfg, HfWaveTerrainCfg) -- same
    integer-pixel arithmetic, int16 elevation grids and [0, 1] normalisation;
  * box sub-terrains, `terrains/primitive_terrains.py:52-376` (BoxFlatTerrainCfg,
    BoxPyramidStairsTerrainCfg, BoxInvertedPyramidStairsTerrainCfg) with the plane / border
    helpers of `terrains/utils.py:11-108`;
  * the grid, `terrains/terrain_generator.py:62-249` (TerrainGenerator: random layout by
    proportion and difficulty, or the curriculum layout -- type per column, difficulty
    rising along rows; patch corners with the grid centred at the origin; spawn origins;
    the 4-box border around the grid), and ROUGH_TERRAINS_CFG (`terrains/config.py:7-57`);
  * the curriculum env origins of `terrains/terrain_importer.py:186-244`.
For the same seed the geoms, sizes, positions and spawn origins are the reference's.

The output is scene data for the compiler (`compiler.model.HFieldSpec` / `BoxSpec`), in
generation order on the static `terrain` body, named terrain_<k> as the reference names
them.  Visual-only parts (colours, materials, lights) are not generated.  A zero-width grid
border adds no boxes (MuJoCo rejects zero-size boxes).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .compiler.model import BoxSpec, HFieldSpec


@dataclass(kw_only=True)
class SubTerrainCfg:
  proportion: float = 1.0
  size: tuple[float, float] = (10.0, 10.0)

  def function(self, difficulty: float, rng: np.random.Generator):
    raise NotImplementedError


def _finish(noise: np.ndarray, size, vertical_scale, base_thickness_ratio, geom_z, spawn_z):
  """Normalise an int16 elevation grid into an hfield (heightfield_terrains.py:195-246)."""
  emin, emax = int(np.min(noise)), int(np.max(noise))
  erange = emax - emin if emax != emin else 1
  max_h = erange * vertical_scale
  base = max_h * base_thickness_ratio
  norm = (noise - emin) / erange if erange > 0 else np.zeros_like(noise, dtype=float)
  hf = dict(size=(size[0] / 2, size[1] / 2, max_h, base), data=norm.astype(np.float32),
            pos=(size[0] / 2, size[1] / 2, geom_z(max_h)))
  origin = np.array([size[0] / 2, size[1] / 2, spawn_z(max_h)])
  return hf, origin


def _check_border(bw, hs):
  if bw > 0 and bw < hs:
    raise ValueError(f"Border width ({bw}) must be >= horizontal scale ({hs})")


@dataclass(kw_only=True)
class HfPyramidSlopedTerrainCfg(SubTerrainCfg):
  """`heightfield_terrains.py:104-246`."""
  slope_range: tuple[float, float]
  platform_width: float = 1.0
  inverted: bool = False
  border_width: float = 0.0
  horizontal_scale: float = 0.1
  vertical_scale: float = 0.005
  base_thickness_ratio: float = 1.0

  def function(self, difficulty, rng):
    if self.inverted:
      slope = -self.slope_range[0] - difficulty * (self.slope_range[1] - self.slope_range[0])
    else:
      slope = self.slope_range[0] + difficulty * (self.slope_range[1] - self.slope_range[0])
    _check_border(self.border_width, self.horizontal_scale)
    hs, vs = self.horizontal_scale, self.vertical_scale
    bp = int(self.border_width / hs)
    wp, lp = int(self.size[0] / hs), int(self.size[1] / hs)
    iw, il = wp - 2 * bp, lp - 2 * bp
    noise = np.zeros((wp, lp), dtype=np.int16)

    def pyramid(w, l, hmax):
      cx, cy = int(w / 2), int(l / 2)
      xx, yy = np.meshgrid(np.arange(0, w), np.arange(0, l), sparse=True)
      xx = ((cx - np.abs(cx - xx)) / cx).reshape(w, 1)
      yy = ((cy - np.abs(cy - yy)) / cy).reshape(1, l)
      raw = hmax * xx * yy
      pw = int(self.platform_width / hs / 2)
      xpf, ypf = w // 2 - pw, l // 2 - pw
      return raw, xpf, ypf

    if bp > 0:
      hmax = int(slope * (iw * hs) / 2 / vs)
      raw, xpf, ypf = pyramid(iw, il, hmax)
      zpf = raw[xpf, ypf] if xpf >= 0 and ypf >= 0 else 0
      raw = np.clip(raw, min(0, zpf), max(0, zpf))
      noise[bp:-bp if bp else wp, bp:-bp if bp else lp] = np.rint(raw).astype(np.int16)
    else:
      hmax = int(slope * self.size[0] / 2 / vs)
      raw, xpf, ypf = pyramid(wp, lp, hmax)
      zpf = raw[xpf, ypf]
      raw = np.clip(raw, min(0, zpf), max(0, zpf))
      noise = np.rint(raw).astype(np.int16)
    inv = self.inverted
    return _finish(noise, self.size, vs, self.base_thickness_ratio,
                   geom_z=lambda h: -h if inv else 0.0,
                   spawn_z=lambda h: -h if inv else h)


@dataclass(kw_only=True)
class HfRandomUniformTerrainCfg(SubTerrainCfg):
  """`heightfield_terrains.py:249-384` (bicubic RectBivariateSpline upsampling)."""
  noise_range: tuple[float, float]
  noise_step: float = 0.005
  downsampled_scale: float | None = None
  horizontal_scale: float = 0.1
  vertical_scale: float = 0.005
  base_thickness_ratio: float = 1.0
  border_width: float = 0.0

  def function(self, difficulty, rng):
    from scipy import interpolate
    _check_border(self.border_width, self.horizontal_scale)
    hs, vs = self.horizontal_scale, self.vertical_scale
    if self.downsampled_scale is None:
      ds = hs
    elif self.downsampled_scale < hs:
      raise ValueError(f"Downsampled scale must be >= horizontal scale: {self.downsampled_scale} < {hs}")
    else:
      ds = self.downsampled_scale
    bp = int(self.border_width / hs)
    wp, lp = int(self.size[0] / hs), int(self.size[1] / hs)
    noise = np.zeros((wp, lp), dtype=np.int16)
    hmin, hmax = int(self.noise_range[0] / vs), int(self.noise_range[1] / vs)
    hstep = int(self.noise_step / vs)
    hrange = np.arange(hmin, hmax + hstep, hstep)

    def field(extent, npx):
      wd, ld = int(extent[0] / ds), int(extent[1] / ds)
      down = rng.choice(hrange, size=(wd, ld))
      f = interpolate.RectBivariateSpline(np.linspace(0, extent[0], wd),
                                          np.linspace(0, extent[1], ld), down)
      return f(np.linspace(0, extent[0], npx[0]), np.linspace(0, extent[1], npx[1]))

    if bp > 0:
      iw, il = wp - 2 * bp, lp - 2 * bp
      z = field((iw * hs, il * hs), (iw, il))
      noise[bp:-bp if bp else wp, bp:-bp if bp else lp] = np.rint(z).astype(np.int16)
    else:
      noise = np.rint(field(self.size, (wp, lp))).astype(np.int16)
    spawn = (self.noise_range[0] + self.noise_range[1]) / 2
    return _finish(noise, self.size, vs, self.base_thickness_ratio,
                   geom_z=lambda h: 0.0, spawn_z=lambda h: spawn)


@dataclass(kw_only=True)
class HfWaveTerrainCfg(SubTerrainCfg):
  """`heightfield_terrains.py:387-499`."""
  amplitude_range: tuple[float, float]
  num_waves: float = 1.0
  horizontal_scale: float = 0.1
  vertical_scale: float = 0.005
  base_thickness_ratio: float = 0.25
  border_width: float = 0.0

  def function(self, difficulty, rng):
    if self.num_waves <= 0:
      raise ValueError(f"Number of waves must be positive. Got: {self.num_waves}")
    _check_border(self.border_width, self.horizontal_scale)
    hs, vs = self.horizontal_scale, self.vertical_scale
    amp = self.amplitude_range[0] + difficulty * (self.amplitude_range[1] - self.amplitude_range[0])
    bp = int(self.border_width / hs)
    wp, lp = int(self.size[0] / hs), int(self.size[1] / hs)
    noise = np.zeros((wp, lp), dtype=np.int16)

    def wave(w, l):
      ap = int(0.5 * amp / vs)
      k = 2 * np.pi / (l / self.num_waves)
      xx, yy = np.meshgrid(np.arange(0, w), np.arange(0, l), sparse=True)
      xx, yy = xx.reshape(w, 1), yy.reshape(1, l)
      return ap * (np.cos(yy * k) + np.sin(xx * k))

    if bp > 0:
      iw, il = wp - 2 * bp, lp - 2 * bp
      noise[bp:-bp if bp else wp, bp:-bp if bp else lp] = np.rint(wave(iw, il)).astype(np.int16)
    else:
      noise = np.rint(wave(wp, lp)).astype(np.int16)
    return _finish(noise, self.size, vs, self.base_thickness_ratio,
                   geom_z=lambda h: -h / 2, spawn_z=lambda h: 0.0)


def _plane_box(size, height, center_zero=True, thickness=1.0):
  """`terrains/utils.py:11-33` make_plane: a finite plane as one box."""
  z = height - thickness / 2.0
  pos = (0.0, 0.0, z) if center_zero else (size[0] / 2.0, size[1] / 2.0, z)
  return [(pos, (size[0] / 2.0, size[1] / 2.0, thickness / 2.0))]


def _border_boxes(size, inner, height, position):
  """`terrains/utils.py:36-108` make_border: top, bottom, left, right boxes around
  `inner` (centred at `position`) out to `size`."""
  tx, ty = (size[0] - inner[0]) / 2.0, (size[1] - inner[1]) / 2.0
  half_tb = (size[0] / 2.0, ty / 2.0, height / 2.0)
  half_lr = (tx / 2.0, inner[1] / 2.0, height / 2.0)
  return [((position[0], position[1] + inner[1] / 2.0 + ty / 2.0, position[2]), half_tb),
          ((position[0], position[1] - inner[1] / 2.0 - ty / 2.0, position[2]), half_tb),
          ((position[0] - inner[0] / 2.0 - tx / 2.0, position[1], position[2]), half_lr),
          ((position[0] + inner[0] / 2.0 + tx / 2.0, position[1], position[2]), half_lr)]


@dataclass(kw_only=True)
class BoxFlatTerrainCfg(SubTerrainCfg):
  """`primitive_terrains.py:52-63`: one 1 m thick box whose top is z = 0."""

  def function(self, difficulty, rng):
    origin = np.array([self.size[0] / 2, self.size[1] / 2, 0.0])
    return _plane_box(self.size, 0.0, center_zero=False), origin


@dataclass(kw_only=True)
class BoxPyramidStairsTerrainCfg(SubTerrainCfg):
  """`primitive_terrains.py:66-222`: rings of 4 boxes climbing to a central platform
  (each step `step_width` wide, `step_height` higher), optional border boxes."""
  border_width: float = 0.0
  step_height_range: tuple[float, float]
  step_width: float
  platform_width: float = 1.0
  holes: bool = False

  def _steps(self, difficulty):
    h = self.step_height_range[0] + difficulty * (self.step_height_range[1] - self.step_height_range[0])
    nx = (self.size[0] - 2 * self.border_width - self.platform_width) // (2 * self.step_width) + 1
    ny = (self.size[1] - 2 * self.border_width - self.platform_width) // (2 * self.step_width) + 1
    return h, int(min(nx, ny))

  def _ring(self, k, tsize, center, box_z, box_height):
    """The 4 boxes of step k: top, bottom (along x), right, left (along y)."""
    sw = self.step_width
    if self.holes:
      bsize = (self.platform_width, self.platform_width)
    else:
      bsize = (tsize[0] - 2 * k * sw, tsize[1] - 2 * k * sw)
    off = (k + 0.5) * sw
    half_x = (bsize[0] / 2.0, sw / 2.0, box_height / 2.0)
    ylen = bsize[1] if self.holes else bsize[1] - 2 * sw
    half_y = (sw / 2.0, ylen / 2.0, box_height / 2.0)
    return [((center[0], center[1] + tsize[1] / 2.0 - off, box_z), half_x),
            ((center[0], center[1] - tsize[1] / 2.0 + off, box_z), half_x),
            ((center[0] + tsize[0] / 2.0 - off, center[1], box_z), half_y),
            ((center[0] - tsize[0] / 2.0 + off, center[1], box_z), half_y)]

  def _border(self, h, z):
    if self.border_width > 0.0 and not self.holes:
      inner = (self.size[0] - 2 * self.border_width, self.size[1] - 2 * self.border_width)
      return _border_boxes(self.size, inner, h, (0.5 * self.size[0], 0.5 * self.size[1], z))
    return []

  def function(self, difficulty, rng):
    h, n = self._steps(difficulty)
    boxes = self._border(h, -h / 2)
    c = (0.5 * self.size[0], 0.5 * self.size[1], 0.0)
    ts = (self.size[0] - 2 * self.border_width, self.size[1] - 2 * self.border_width)
    for k in range(n):
      boxes += self._ring(k, ts, c, c[2] + k * h / 2.0, (k + 2) * h)
    sw = self.step_width
    boxes.append(((c[0], c[1], c[2] + n * h / 2),
                  ((ts[0] - 2 * n * sw) / 2.0, (ts[1] - 2 * n * sw) / 2.0, (n + 2) * h / 2.0)))
    return boxes, np.array([c[0], c[1], (n + 1) * h])


@dataclass(kw_only=True)
class BoxInvertedPyramidStairsTerrainCfg(BoxPyramidStairsTerrainCfg):
  """`primitive_terrains.py:225-376`: the same rings stepping down into a pit."""

  def function(self, difficulty, rng):
    h, n = self._steps(difficulty)
    total = (n + 1) * h
    boxes = self._border(h, -0.5 * h)
    c = (0.5 * self.size[0], 0.5 * self.size[1], 0.0)
    ts = (self.size[0] - 2 * self.border_width, self.size[1] - 2 * self.border_width)
    for k in range(n):
      boxes += self._ring(k, ts, c, c[2] - total / 2 - (k + 1) * h / 2.0, total - (k + 1) * h)
    sw = self.step_width
    boxes.append(((c[0], c[1], c[2] - total - h / 2),
                  ((ts[0] - 2 * n * sw) / 2.0, (ts[1] - 2 * n * sw) / 2.0, h / 2.0)))
    return boxes, np.array([c[0], c[1], -(n + 1) * h])


@dataclass(kw_only=True)
class TerrainGeneratorCfg:
  """`terrain_generator.py:50-64`."""
  seed: int | None = None
  curriculum: bool = False
  size: tuple[float, float]
  border_width: float = 0.0
  border_height: float = 1.0
  num_rows: int = 1
  num_cols: int = 1
  sub_terrains: dict[str, SubTerrainCfg] = field(default_factory=dict)
  difficulty_range: tuple[float, float] = (0.0, 1.0)


@dataclass
class TerrainImporterCfg:
  """`terrains/terrain_importer.py:30-60`: a plane (env origins on a grid of `env_spacing`)
  or a generated terrain (`terrain_generator`, env origins from its sub-terrain spawn points
  with the curriculum's initial levels up to `max_init_terrain_level`)."""
  terrain_type: str = "plane"
  terrain_generator: TerrainGeneratorCfg | None = None
  env_spacing: float | None = 2.0
  max_init_terrain_level: int | None = None
  num_envs: int = 1


class TerrainGenerator:
  """`terrain_generator.py:62-249`: patch grid centred at the origin; random layout
  (per-patch proportion draw + uniform difficulty) or curriculum layout (type per column,
  difficulty rising along rows), then the border boxes.  `generate()` returns the terrain
  geoms (HFieldSpec / BoxSpec, world positions, generation order) and the
  [num_rows, num_cols, 3] spawn origins."""

  def __init__(self, cfg: TerrainGeneratorCfg):
    if len(cfg.sub_terrains) == 0:
      raise ValueError("At least one sub_terrain must be specified.")
    self.cfg = cfg
    for sub in cfg.sub_terrains.values():
      sub.size = cfg.size
    seed = cfg.seed if cfg.seed is not None else np.random.randint(0, 10000)
    self.np_rng = np.random.default_rng(seed)
    self.terrain_origins = np.zeros((cfg.num_rows, cfg.num_cols, 3))
    self.geoms: list = []

  @property
  def hfields(self) -> list[HFieldSpec]:
    return [g for g in self.geoms if isinstance(g, HFieldSpec)]

  def _position(self, row, col):
    c = self.cfg
    return np.array([-c.num_rows * c.size[0] * 0.5 + row * c.size[0],
                     -c.num_cols * c.size[1] * 0.5 + col * c.size[1], 0.0])

  def _name(self):
    return f"terrain_{len(self.geoms)}"

  def _create(self, world_position, difficulty, sub):
    out, origin = sub.function(difficulty, self.np_rng)
    if isinstance(out, dict):  # one heightfield
      pos = tuple(float(v) for v in np.asarray(out["pos"]) + world_position)
      self.geoms.append(HFieldSpec(name=self._name(), pos=pos,
                                   size=tuple(float(v) for v in out["size"]), data=out["data"]))
    else:  # boxes: (local position, half sizes)
      for pos, half in out:
        self.geoms.append(BoxSpec(name=self._name(),
                                  pos=tuple(float(v) for v in np.asarray(pos, float) + world_position),
                                  size=tuple(float(v) for v in half)))
    return origin + world_position

  def _border(self):
    """`terrain_generator.py:225-248`: 4 boxes around the grid, top at z = 0."""
    c = self.cfg
    if c.border_width <= 0:
      return
    inner = (c.num_rows * c.size[0], c.num_cols * c.size[1])
    outer = (inner[0] + 2 * c.border_width, inner[1] + 2 * c.border_width)
    for pos, half in _border_boxes(outer, inner, abs(c.border_height), (0, 0, -c.border_height / 2)):
      self.geoms.append(BoxSpec(name=self._name(), pos=tuple(float(v) for v in pos),
                                size=tuple(float(v) for v in half)))

  def generate(self):
    c = self.cfg
    props = np.array([s.proportion for s in c.sub_terrains.values()], dtype=float)
    props /= np.sum(props)
    subs = list(c.sub_terrains.values())
    if c.curriculum:
      idx = [int(np.min(np.where(i / c.num_cols + 0.001 < np.cumsum(props))[0]))
             for i in range(c.num_cols)]
      for col in range(c.num_cols):
        for row in range(c.num_rows):
          lo, hi = c.difficulty_range
          diff = lo + (hi - lo) * (row + self.np_rng.uniform()) / c.num_rows
          self.terrain_origins[row, col] = self._create(self._position(row, col), diff, subs[idx[col]])
    else:
      for index in range(c.num_rows * c.num_cols):
        row, col = (int(v) for v in np.unravel_index(index, (c.num_rows, c.num_cols)))
        si = self.np_rng.choice(len(props), p=props)
        diff = self.np_rng.uniform(*c.difficulty_range)
        self.terrain_origins[row, col] = self._create(self._position(row, col), diff, subs[si])
    self._border()
    return self.geoms, self.terrain_origins


def rough_terrains_cfg(seed: int | None = None, curriculum: bool = False, num_rows: int = 10,
                       num_cols: int = 20, border_width: float = 20.0) -> TerrainGeneratorCfg:
  """ROUGH_TERRAINS_CFG (`terrains/config.py:7-57`): 8 m x 8 m patches, 10 x 20 grid, 20 m
  border; 40% flat boxes, 30% pyramid stairs, 30% inverted pyramid stairs (its heightfield
  entries are commented out in the reference).  Play mode
  (`tasks/velocity/config/{g1,go1}/env_cfgs.py`, play overrides) asks for the random layout
  (curriculum off) on a 5 x 5 grid with a 10 m border."""
  stairs = dict(step_height_range=(0.0, 0.1), step_width=0.3, platform_width=3.0, border_width=1.0)
  return TerrainGeneratorCfg(
    seed=seed, curriculum=curriculum, size=(8.0, 8.0), border_width=border_width,
    num_rows=num_rows, num_cols=num_cols,
    sub_terrains={
      "flat": BoxFlatTerrainCfg(proportion=0.4),
      "pyramid_stairs": BoxPyramidStairsTerrainCfg(proportion=0.3, **stairs),
      "pyramid_stairs_inv": BoxInvertedPyramidStairsTerrainCfg(proportion=0.3, **stairs),
    })


def hf_rough_terrains_cfg(seed: int = 0) -> TerrainGeneratorCfg:
  """Config-5 terrain: the reference's heightfield sub-terrains, commented
  out of ROUGH_TERRAINS_CFG in `terrains/config.py:28-54`, on its 8 m x 8 m, 10 x 20
  patch grid, seeded, without the border."""
  return TerrainGeneratorCfg(
    seed=seed, size=(8.0, 8.0), num_rows=10, num_cols=20,
    sub_terrains={
      "hf_pyramid_slope": HfPyramidSlopedTerrainCfg(proportion=0.1, slope_range=(0.0, 1.0),
                                                    platform_width=2.0, border_width=0.25),
      "hf_pyramid_slope_inv": HfPyramidSlopedTerrainCfg(proportion=0.1, slope_range=(0.0, 1.0),
                                                        platform_width=2.0, border_width=0.25,
                                                        inverted=True),
      "random_rough": HfRandomUniformTerrainCfg(proportion=0.2, noise_range=(0.02, 0.10),
                                                noise_step=0.02, border_width=0.25),
      "wave_terrain": HfWaveTerrainCfg(proportion=0.2, amplitude_range=(0.0, 0.2), num_waves=4,
                                       border_width=0.25),
    })


def curriculum_env_origins(terrain_origins, num_envs: int, max_init_terrain_level=None,
                           generator=None):
  """`terrain_importer.py:224-244`: random level (row) per env, type (column) by env
  index block.  Returns (env_origins [N,3], levels [N], types [N]) as numpy."""
  import torch
  origins = torch.as_tensor(terrain_origins, dtype=torch.float32)
  nrows, ncols = origins.shape[:2]
  max_init = nrows - 1 if max_init_terrain_level is None else min(max_init_terrain_level, nrows - 1)
  levels = torch.randint(0, max_init + 1, (num_envs,), generator=generator)
  types = torch.div(torch.arange(num_envs), (num_envs / ncols), rounding_mode="floor").to(torch.long)
  return origins[levels, types], levels, types
