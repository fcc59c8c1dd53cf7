import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def golden_dir():
    return ROOT / "tests" / "golden"


@pytest.fixture(autouse=True)
def _no_device_fault():
    """Every GPU test: no list guard may fire in any context it closes
    (yastack_amd.abi.FAULT_LOG, filled by SoftRss.close from the context's
    fault record), whether or not the test reads yrss_status itself."""
    try:
        from yastack_amd import abi
    except Exception:   # pragma: no cover - import errors surface in the test itself
        yield
        return
    abi.FAULT_LOG.clear()
    yield
    assert not abi.FAULT_LOG, f"device guard fired: {abi.FAULT_LOG}"
