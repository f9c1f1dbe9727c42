"""Multi-GPU path logic on the CPU: shard ranges, outcome packing and the
gather to rank 0 (gloo, world_size 2, two processes), against one unsharded run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from fast_kinematic_simulator_amd.sharding import pack_outcomes, shard_bounds, unpack_outcomes

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("n,world", [(13, 2), (65536, 8), (7, 8), (0, 2), (1048576, 3)])
def test_shard_bounds_cover_the_batch(n, world):
    ranges = [shard_bounds(n, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(ranges[r][1] == ranges[r + 1][0] for r in range(world - 1))
    sizes = [b - a for a, b in ranges]
    assert max(sizes) - min(sizes) <= 1 and sizes[0] == max(sizes)


def test_pack_roundtrip():
    rng = np.random.default_rng(0)
    q = rng.normal(size=(5, 7))
    col = np.array([1, 0, 1, 0, 0], dtype=np.uint8)
    micro = np.array([3, 4000000000, 7, 0, 1], dtype=np.uint32)
    res = np.array([0, 25, 3, 0, 1], dtype=np.uint32)
    err = np.array([0, 0x80, 0, 0x1, 0], dtype=np.uint32)
    u = unpack_outcomes(pack_outcomes(q, col, micro, res, err))
    assert np.array_equal(u["positions"], q)
    assert np.array_equal(u["collided"], col.astype(bool))
    assert np.array_equal(u["microsteps"], micro) and np.array_equal(u["resolver_iterations"], res)
    assert np.array_equal(u["error_flags"], err)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_world2_gather_matches_single_run(oracle_lib, tmp_path):
    port = _free_port()
    out = tmp_path / "verdict.json"
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "gloo_shard_worker.py"), "--rank", str(r), "--world", "2",
                               "--port", str(port), "--out", str(out)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              env=dict(os.environ, OMP_NUM_THREADS="1"))
             for r in range(2)]
    logs = [p.communicate(timeout=240)[0].decode() for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    v = json.loads(out.read_text())
    assert v["rows"] == 13 and v["identical"], v
    assert v["collided"] > 0


def test_c_shard_bounds_match_python(fks_lib):
    """fks_shard_bounds (the multi-device context's split) is sharding.shard_bounds."""
    import ctypes

    from fast_kinematic_simulator_amd.sharding import shard_bounds

    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    for n in (0, 1, 7, 64, 65536, 1048577, 2 ** 40 + 3):
        for world in (1, 2, 3, 8, 13):
            prev = 0
            for r in range(world):
                assert fks_lib.fks_shard_bounds(n, world, r, ctypes.byref(lo), ctypes.byref(hi)) == 0
                assert (lo.value, hi.value) == shard_bounds(n, world, r)
                assert lo.value == prev
                prev = hi.value
            assert prev == n
    assert fks_lib.fks_shard_bounds(4, 0, 0, ctypes.byref(lo), ctypes.byref(hi)) == 1
    assert fks_lib.fks_shard_bounds(4, 2, 2, ctypes.byref(lo), ctypes.byref(hi)) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_context_matches_single(fks_lib, oracle_lib, devices):
    """fks_create_multi over a device list (the same MI355X listed k times runs k shards on
    k contexts): results bit-identical to one context and to the oracle; statistics summed."""
    import oracle
    from fast_kinematic_simulator_amd import MultiDeviceSimulator, make_linked_simulator
    from fast_kinematic_simulator_amd import workloads as W

    wl = W.cfg3(61 / 65536)
    multi = MultiDeviceSimulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed, devices)
    single = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        assert multi.num_devices() == len(devices)
        multi.set_call_index(3)
        single.set_call_index(3)
        m = multi.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        s = single.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
            assert np.array_equal(m[k], s[k]), k
        assert multi.get_statistics() == single.get_statistics()
        mc, sc = multi.last_call_counters(), single.last_call_counters()
        for k in ("particles", "microsteps", "resolver_iterations", "sdf_bytes", "least_squares_rows", "controller_steps"):
            assert mc[k] == sc[k], k
    finally:
        multi.close()
        single.close()
    o = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True,
                                call_index=3)
    assert np.array_equal(m["positions"], o["positions"])


@pytest.mark.gpu
def test_multi_device_context_over_every_visible_gpu(fks_lib, oracle_lib):
    """fks_create_multi over every visible MI355X (one shard per physical device): results
    bit-identical to one context and to the oracle, statistics summed (skips below 2 GPUs)."""
    import torch

    import oracle
    from fast_kinematic_simulator_amd import MultiDeviceSimulator, make_linked_simulator
    from fast_kinematic_simulator_amd import workloads as W

    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs 2 or more GPUs")
    wl = W.cfg3((16 * n + 3) / 65536)
    multi = MultiDeviceSimulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed, list(range(n)))
    single = make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed)
    try:
        assert multi.num_devices() == n
        multi.set_call_index(5)
        single.set_call_index(5)
        m = multi.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        s = single.forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
        for k in ("positions", "collided", "microsteps", "resolver_iterations", "error_flags"):
            assert np.array_equal(m[k], s[k]), k
        assert multi.get_statistics() == single.get_statistics()
    finally:
        multi.close()
        single.close()
    o = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts, wl.targets, True,
                                call_index=5)
    assert np.array_equal(m["positions"], o["positions"]) and np.array_equal(m["microsteps"], o["microsteps"])


@pytest.mark.gpu
def test_two_contexts_on_two_streams_overlap_without_changing_results(fks_lib, oracle_lib):
    """Consecutive batches alternated over two contexts on two streams (bench.py's
    `pipelined` figure): each enqueue returns at once, the batches may run concurrently, and
    every batch's outcomes equal a sequential call at the same RNG call index bit for bit
    (and the oracle's for the first)."""
    import torch

    import oracle
    from fast_kinematic_simulator_amd import make_linked_simulator
    from fast_kinematic_simulator_amd import workloads as W

    wl = W.cfg3(3000 / 65536)  # more particles than one wave slot each: segments in play
    dev = torch.device("cuda", 0)
    n, Wd = wl.starts.shape[0], wl.robot.config_width
    sims = [make_linked_simulator(wl.environment(), wl.solver, wl.controller_frequency, wl.seed) for _ in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    starts = torch.from_numpy(np.ascontiguousarray(wl.starts)).to(dev)
    targets = torch.from_numpy(np.ascontiguousarray(wl.targets)).to(dev)
    batches = 4
    outs = [[torch.empty((n, Wd), dtype=torch.float64, device=dev), torch.empty(n, dtype=torch.uint8, device=dev),
             torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
             torch.empty(n, dtype=torch.int32, device=dev)] for _ in range(batches)]
    try:
        for s in sims:
            s.set_robot(wl.robot)
        torch.cuda.synchronize()
        for k in range(batches):
            j = k % 2
            sims[j].set_call_index(k)
            q, c, m, r, e = outs[k]
            sims[j].forward_simulate_device(wl.robot, starts.data_ptr(), n, targets.data_ptr(), 1, 0, True, q.data_ptr(),
                                            c.data_ptr(), m.data_ptr(), r.data_ptr(), e.data_ptr(),
                                            stream=streams[j].cuda_stream, synchronize=False)
        torch.cuda.synchronize()
        for k in range(batches):
            sims[0].set_call_index(k)
            ref = sims[0].forward_simulate_arrays(wl.robot, wl.starts, wl.targets, True)
            got = [t.cpu().numpy() for t in outs[k]]
            assert np.array_equal(got[0], ref["positions"]), k
            assert np.array_equal(got[1].astype(bool), ref["collided"]), k
            assert np.array_equal(got[2].astype(np.uint32), ref["microsteps"]), k
            assert np.array_equal(got[3].astype(np.uint32), ref["resolver_iterations"]), k
            assert np.array_equal(got[4].astype(np.uint32), ref["error_flags"]), k
    finally:
        for s in sims:
            s.close()
    o = oracle.forward_simulate(wl.environment(), wl.robot, wl.solver, wl.controller_frequency, wl.seed, wl.starts[:256],
                                wl.targets, True, call_index=0)
    assert np.array_equal(outs[0][0].cpu().numpy()[:256], o["positions"])
