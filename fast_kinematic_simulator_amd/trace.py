"""ForwardSimulationStepTrace on the host side of the C-ABI.

The reference fills a nested trace while it simulates one particle with
``enable_tracing = true`` (SPCS:1583-1588 adds a resolver step per controller
step, SPCS:1593 a contact-resolver step per microstep, SPCS:1615-1618,
1701-1704, 1712-1715 and 1776-1779 push configurations).  The HIP path writes
the same records flat, per particle, into ``fks_trace`` buffers
(include/fks_capi.h); this module allocates those buffers and rebuilds the
nested structure from them.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List

import numpy as np

from . import _capi

TRACE_POST_ACTION = 0     # post_action_configuration of a microstep (SPCS:1617)
TRACE_RESOLVER_STEP = 1   # active_configuration after a resolver iteration (SPCS:1703)
TRACE_RESOLVE_FAILED = 2  # previous_configuration, resolver gave up (SPCS:1714)
TRACE_CONTACT_STOP = 3    # previous_configuration, contact with allow_contacts == false (SPCS:1778)


@dataclass
class ForwardSimulationContactResolverStepTrace:
    """One microstep: the configurations pushed while it ran."""
    contact_resolution_steps: List[np.ndarray] = field(default_factory=list)
    kinds: List[int] = field(default_factory=list)


@dataclass
class ForwardSimulationResolverTrace:
    """One controller step (SPCS:1583-1588)."""
    control_input: np.ndarray
    control_input_step: np.ndarray
    number_microsteps: int
    contact_resolver_steps: List[ForwardSimulationContactResolverStepTrace] = field(default_factory=list)


@dataclass
class ForwardSimulationStepTrace:
    resolver_steps: List[ForwardSimulationResolverTrace] = field(default_factory=list)
    truncated: bool = False  # records beyond the buffer capacities were dropped


class TraceBuffers:
    """Caller-owned host buffers of one traced call (fks_trace)."""

    def __init__(self, n: int, num_dofs: int, config_width: int, step_capacity: int, config_capacity: int):
        self.n, self.D, self.W = int(n), int(num_dofs), int(config_width)
        self.step_capacity, self.config_capacity = int(step_capacity), int(config_capacity)
        self.step_inputs = np.zeros((self.n, self.step_capacity, 2, self.D), dtype=np.float64)
        self.step_microsteps = np.zeros((self.n, self.step_capacity), dtype=np.uint32)
        self.configs = np.zeros((self.n, self.config_capacity, self.W), dtype=np.float64)
        self.config_tags = np.zeros((self.n, self.config_capacity, 3), dtype=np.uint32)
        self.num_steps = np.zeros(self.n, dtype=np.uint32)
        self.num_configs = np.zeros(self.n, dtype=np.uint32)

    def to_c(self) -> _capi.Trace:
        t = _capi.Trace()
        t.step_capacity = self.step_capacity
        t.config_capacity = self.config_capacity
        t.step_inputs = _capi.as_ptr(self.step_inputs, ctypes.c_double)
        t.step_microsteps = _capi.as_ptr(self.step_microsteps, ctypes.c_uint32)
        t.configs = _capi.as_ptr(self.configs, ctypes.c_double)
        t.config_tags = _capi.as_ptr(self.config_tags, ctypes.c_uint32)
        t.num_steps = _capi.as_ptr(self.num_steps, ctypes.c_uint32)
        t.num_configs = _capi.as_ptr(self.num_configs, ctypes.c_uint32)
        return t

    def particle(self, i: int) -> ForwardSimulationStepTrace:
        """Nested trace of particle i (records are grouped by their (step, microstep) tags)."""
        ns, nc = int(self.num_steps[i]), int(self.num_configs[i])
        tr = ForwardSimulationStepTrace(truncated=ns > self.step_capacity or nc > self.config_capacity)
        for k in range(min(ns, self.step_capacity)):
            tr.resolver_steps.append(ForwardSimulationResolverTrace(
                self.step_inputs[i, k, 0].copy(), self.step_inputs[i, k, 1].copy(), int(self.step_microsteps[i, k])))
        last = None
        for k in range(min(nc, self.config_capacity)):
            step, micro, kind = (int(v) for v in self.config_tags[i, k])
            if step >= len(tr.resolver_steps):
                break
            rs = tr.resolver_steps[step]
            if last != (step, micro):
                rs.contact_resolver_steps.append(ForwardSimulationContactResolverStepTrace())
                last = (step, micro)
            rs.contact_resolver_steps[-1].contact_resolution_steps.append(self.configs[i, k].copy())
            rs.contact_resolver_steps[-1].kinds.append(kind)
        return tr

    def traces(self) -> List[ForwardSimulationStepTrace]:
        return [self.particle(i) for i in range(self.n)]
