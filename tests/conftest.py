import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity of the HIP path against the CPU oracle")


@pytest.fixture(scope="session")
def fks_lib():
    from fast_kinematic_simulator_amd.build import build_library
    from fast_kinematic_simulator_amd import _capi

    build_library()
    # torch bundles its own HIP runtime; it must initialise before libfks_hip.so's
    # (/opt/rocm) runtime opens the device, as bench.py does, or torch finds no GPU
    try:
        import torch

        if torch.cuda.is_available():
            torch.zeros(1, device="cuda:0")
    except ImportError:
        pass
    return _capi.lib()


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle

    oracle.build()
    return oracle.lib()
