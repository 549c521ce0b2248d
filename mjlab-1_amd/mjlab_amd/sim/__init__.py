from .sim import (MujocoCfg, NanGuard, NanGuardCfg, Simulation, SimulationCfg, load_nan_dump,
                  world_capacity)
from .sim_data import DeviceBridge, WarpBridge

__all__ = ["MujocoCfg", "NanGuard", "NanGuardCfg", "load_nan_dump", "Simulation", "SimulationCfg", "DeviceBridge",
           "WarpBridge", "world_capacity"]
