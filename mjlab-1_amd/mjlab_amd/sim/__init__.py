from .sim import MujocoCfg, NanGuardCfg, Simulation, SimulationCfg, world_capacity
from .sim_data import DeviceBridge, WarpBridge

__all__ = ["MujocoCfg", "NanGuardCfg", "Simulation", "SimulationCfg", "DeviceBridge",
           "WarpBridge", "world_capacity"]
