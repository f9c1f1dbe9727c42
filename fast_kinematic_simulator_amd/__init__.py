"""MI355X-native particle forward-simulation path of fast_kinematic_simulator.

The hot path (ForwardSimulateRobots -> ForwardSimulateMutableRobot ->
ResolveForwardSimulation, reference simple_particle_contact_simulator.hpp) runs
as hand-written HIP kernels for gfx950 behind the C-ABI in include/fks_capi.h.
"""
from ._capi import FksError, lib
from .environment import (DeviceEnvironment, ObstacleConfig, SimulatorEnvironment, build_complete_environment,
                          build_device_environment)
from .robots import (ControllerConfig, Joint, RobotDescription, SampledActuatorModel, make_linked_robot,
                     make_sampled_actuator_model, make_se2_robot, make_se3_robot, se3_pose, transform34)
from .simulator import (HipParticleContactSimulator, MultiDeviceSimulator, SimulationResult, SimulatorSolverParameters,
                        get_default_solver_parameters, make_linked_simulator, make_se2_simulator, make_se3_simulator)

__all__ = [
    "FksError", "lib", "ObstacleConfig", "SimulatorEnvironment", "build_complete_environment", "ControllerConfig", "Joint",
    "RobotDescription", "make_linked_robot", "make_se2_robot", "make_se3_robot", "se3_pose", "transform34",
    "HipParticleContactSimulator", "MultiDeviceSimulator", "SimulationResult", "SimulatorSolverParameters", "get_default_solver_parameters",
    "make_linked_simulator", "make_se2_simulator", "make_se3_simulator",
]
