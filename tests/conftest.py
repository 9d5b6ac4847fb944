import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native():
    """The native module; built on demand so a fresh checkout can test."""
    try:
        from accel_sim_framework_distributed_amd import _native
        return _native.load()
    except ImportError:
        import build_native
        build_native.build(cpu_only=False, extra=False)
        from accel_sim_framework_distributed_amd import _native
        return _native.load()


@pytest.fixture(scope="session")
def qv100_args():
    from accel_sim_framework_distributed_amd.models import presets
    return presets.args_for("QV100")


@pytest.fixture(scope="session")
def tmpdir_session(tmp_path_factory):
    return tmp_path_factory.mktemp("asim")


def reference_path(*parts):
    p = os.path.join(REFERENCE, *parts)
    return p if os.path.exists(p) else None
