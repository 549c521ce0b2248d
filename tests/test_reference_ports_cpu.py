"""The CPU-side halves of the reference's sensor / bridge tests (no physics): the builtin
sensor cfg's object-type rules (`tests/test_builtin_sensor.py:191-268,307-327`) and the
device bridge's attribute refusal (`tests/test_sim_data.py:67-75`)."""

import pytest
import torch

from mjlab_amd.entity import EntityCfg
from mjlab_amd.scene import Scene, SceneCfg
from mjlab_amd.sensor import BuiltinSensorCfg, ObjRef
from mjlab_amd.spec import Spec

ROBOT_WITH_XML_SENSORS = """
    <mujoco>
      <worldbody>
        <body name="base" pos="0 0 1">
          <freejoint name="free_joint"/>
          <geom name="base_geom" type="box" size="0.2 0.2 0.1" mass="5.0"/>
          <site name="base_site" pos="0 0 0"/>
          <body name="link1" pos="0.3 0 0">
            <joint name="joint1" type="hinge" axis="0 0 1" range="-1.57 1.57"/>
            <geom name="link1_geom" type="box" size="0.1 0.1 0.1" mass="1.0"/>
            <site name="link1_site" pos="0 0 0"/>
          </body>
        </body>
      </worldbody>
      <sensor>
        <jointpos name="xml_joint_sensor" joint="joint1"/>
        <accelerometer name="xml_accel_sensor" site="base_site"/>
        <gyro name="xml_gyro_sensor" site="link1_site"/>
      </sensor>
    </mujoco>
"""


def test_error_on_invalid_ref():
  with pytest.raises(ValueError, match="does not support ref specification"):
    BuiltinSensorCfg(name="invalid_sensor", sensor_type="jointpos",
                     obj=ObjRef(type="joint", name="joint1", entity="robot"),
                     ref=ObjRef(type="body", name="base"))


def test_error_on_missing_obj():
  with pytest.raises(ValueError, match="requires obj with type='joint'"):
    BuiltinSensorCfg(name="invalid_sensor", sensor_type="jointpos")


def test_error_on_wrong_obj_type_for_site_sensor():
  with pytest.raises(ValueError, match="requires obj.type='site'"):
    BuiltinSensorCfg(name="invalid_sensor", sensor_type="accelerometer", obj=ObjRef(type="body", name="base"))


def test_error_on_wrong_obj_type_for_body_sensor():
  with pytest.raises(ValueError, match="requires obj.type='body'"):
    BuiltinSensorCfg(name="invalid_sensor", sensor_type="subtreecom", obj=ObjRef(type="site", name="base"))


def test_error_on_wrong_obj_type_for_joint_sensor():
  with pytest.raises(ValueError, match="requires obj.type='joint'"):
    BuiltinSensorCfg(name="invalid_sensor", sensor_type="jointvel", obj=ObjRef(type="body", name="base"))


def test_spatial_frame_sensor_accepts_multiple_types():
  for t in ("body", "xbody", "geom", "site", "camera"):
    BuiltinSensorCfg(name=f"frame_sensor_{t}", sensor_type="framepos", obj=ObjRef(type=t, name="test"))


def test_builtin_sensor_errors_on_duplicate_name():
  entity_cfg = EntityCfg(spec_fn=lambda: Spec.from_string(ROBOT_WITH_XML_SENSORS))
  dup = BuiltinSensorCfg(name="xml_joint_sensor", sensor_type="jointpos",
                         obj=ObjRef(type="joint", name="joint1", entity="robot"))
  scene_cfg = SceneCfg(num_envs=2, env_spacing=3.0, entities={"robot": entity_cfg}, sensors=(dup,))
  with pytest.raises(ValueError, match="defined in both entity XML and scene config"):
    Scene(scene_cfg, "cpu")


def test_builtin_sensor_cfg_compiles():
  """A scene-config sensor lands in the compiled model after the entity's XML sensors."""
  entity_cfg = EntityCfg(spec_fn=lambda: Spec.from_string(ROBOT_WITH_XML_SENSORS))
  extra = BuiltinSensorCfg(name="link_vel", sensor_type="jointvel",
                           obj=ObjRef(type="joint", name="joint1", entity="robot"))
  m = Scene(SceneCfg(num_envs=1, entities={"robot": entity_cfg}, sensors=(extra,)), "cpu").compile()
  assert m.names["sensor"] == ["robot/xml_joint_sensor", "robot/xml_accel_sensor",
                               "robot/xml_gyro_sensor", "robot/link_vel"]
  assert m.nsensordata == 1 + 3 + 3 + 1


def test_bridge_raises_on_setattr():
  from mjlab_amd.sim.sim_data import WarpBridge
  bridge = WarpBridge(object())
  with pytest.raises(AttributeError, match="Cannot set attribute 'arr' on WarpBridge"):
    bridge.arr = torch.zeros((2, 2))
  with pytest.raises(AttributeError, match="Use in-place operations instead"):
    bridge.val = 42.0
