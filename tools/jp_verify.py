"""Joint-space proof verification (FKS_VERIFY_JP build, FKS_LIB_PATH=...): every microstep
the proof settles is also FK'd and checked in full; a disagreement ends the particle with
bit 30 (environment) / bit 29 (self-collision) in its error flags.  Prints the counts and
the first offending particles.

    FKS_LIB_PATH=build/variants/libfks_verify.so python tools/jp_verify.py cfg3 4096
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fast_kinematic_simulator_amd import make_linked_simulator  # noqa: E402
from fast_kinematic_simulator_amd import workloads as W  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    base = {"cfg1": 32, "cfg2": 4096, "cfg3": 65536, "cfg4": 1048576, "cfg5": 1048576}.get(name, 1)
    wl = W.WORKLOADS[name](n / float(base))
    sim = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    sim.set_joint_proof(True)
    if len(sys.argv) > 3:
        sim.set_segment_steps(int(sys.argv[3]))
    out = sim.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, wl.allow_contacts)
    c = sim.last_call_counters()
    sim.close()
    err = np.asarray(out["error_flags"], dtype=np.uint64)
    env = np.nonzero(err & (1 << 30))[0]
    slf = np.nonzero(err & (1 << 29))[0]
    print(json.dumps({"workload": name, "particles": int(len(err)), "segment_steps": sys.argv[3] if len(sys.argv) > 3 else None, "env_violations": int(len(env)),
                      "self_violations": int(len(slf)), "first_env": env[:8].tolist(), "first_self": slf[:8].tolist(),
                      "micro_at_stop": [int(out["microsteps"][i]) for i in env[:8]],
                      "error_flags": {hex(int(k)): int(v) for k, v in zip(*np.unique(err, return_counts=True))},
                      "proven": c["proven_free_microsteps"], "microsteps": c["microsteps"]}))


if __name__ == "__main__":
    main()
