import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "fibsem-optflow_amd"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def built():
    """Ensure native artefacts exist (build once per session if missing)."""
    from optflow_amd import capi
    from oracle import checker
    if not capi.ENGINE_SO.exists() or not checker.ORACLE_SO.exists():
        import __graft_entry__
        __graft_entry__.build()
    return True
