"""Regenerate tests/golden/pid_trace_golden.json: a simulated trajectory's PID inputs
run through the reference's own PID header.

The oracle traces workloads.pid_free_space (free space, actuator noise bounds 0, PID
term inside the velocity clamp).  The error each controller step feeds the PID is
target - q_k (GenerateControlAction, TNUVA:598-614), where q_k is the configuration the
step starts from (the start, then the last configuration of the previous step).  Those
sequences, per particle and dof, go through oracle/_ref/pid_golden --replay, which
compiles /root/reference/include/fast_kinematic_simulator/simple_pid_controller.hpp
where it lies (oracle/Makefile `ref`).  The fixture holds the errors, dt, the
reference's ComputeFeedbackTerm outputs and the velocity limits, all as hex floats.
Needs /root/reference (this container only); the tests read the fixture."""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def step_errors(starts, targets, buf, steps):
    """errors[i, k, d] = target - q_k per particle from a TraceBuffers of the run."""
    n, D = starts.shape
    err = np.zeros((n, steps, D))
    for i in range(n):
        tr = buf.particle(i)
        assert len(tr.resolver_steps) == steps, "every particle runs every controller step"
        q = starts[i].copy()
        for k, rs in enumerate(tr.resolver_steps):
            err[i, k] = targets[0] - q
            kinds = [kd for c in rs.contact_resolver_steps for kd in c.kinds]
            assert all(kd == 0 for kd in kinds), "free space: post-action configurations only"
            q = rs.contact_resolver_steps[-1].contact_resolution_steps[-1].copy()
    return err


def main():
    import oracle
    from fast_kinematic_simulator_amd import workloads as W

    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, stdout=subprocess.DEVNULL)
    wl = W.pid_free_space()
    r, buf = oracle.forward_simulate_traced(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts,
                                            wl.targets, True)
    dt = 1.0 / wl.controller_frequency
    err = step_errors(wl.starts, wl.targets, buf, wl.steps)
    n, T, D = err.shape
    lines = []
    for i in range(n):
        for d in range(D):
            c = wl.robot.controllers[d]
            lines.append(f"{float(c.kp).hex()} {float(c.ki).hex()} {float(c.kd).hex()} {float(c.integral_clamp).hex()} {T}")
            lines += [f"{float(err[i, k, d]).hex()} {float(dt).hex()}" for k in range(T)]
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "pid_golden"), "--replay"], input="\n".join(lines) + "\n",
                         capture_output=True, text=True, check=True).stdout.split()
    terms = np.array([float.fromhex(v) for v in out]).reshape(n, D, T).transpose(0, 2, 1)
    vmax = np.array([abs(c.velocity_limit) for c in wl.robot.controllers])
    assert np.all(np.abs(terms) < vmax), "the scene keeps the PID term inside the velocity clamp"
    golden = {"source": "reference simple_pid_controller.hpp via oracle/_ref/pid_golden --replay "
                        "(tests/golden/make_pid_trace_golden.py)",
              "workload": wl.name, "dt": dt.hex(), "velocity_limits": [float(v).hex() for v in vmax],
              "errors": [[[float(v).hex() for v in row] for row in p] for p in err],
              "pid_terms": [[[float(v).hex() for v in row] for row in p] for p in terms]}
    with open(os.path.join(HERE, "pid_trace_golden.json"), "w") as f:
        json.dump(golden, f)
    print("wrote", os.path.join(HERE, "pid_trace_golden.json"), f"({n} particles x {T} steps x {D} dofs)")


if __name__ == "__main__":
    main()
