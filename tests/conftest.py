import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slurm-bridge-operator_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "auto_engine: keep the production engine choice (small batches "
                                       "on the host-driven rounds) instead of forcing the persistent engine")


@pytest.fixture(autouse=True)
def _persistent_engine_by_default(request, monkeypatch):
    """GPU parity tests exercise the persistent engine at every size: the production default sends
    placements of <= FIT_SMALL_BATCH live jobs to the host-driven rounds (engine.cpp small_batch),
    which would move most small parity cases off the engine they were written for.  Tests that set
    FIT_ENGINE themselves override this; `auto_engine` tests (admission) keep the default."""
    if request.node.get_closest_marker("gpu") and not request.node.get_closest_marker("auto_engine") \
            and "FIT_ENGINE" not in os.environ:
        monkeypatch.setenv("FIT_ENGINE", "persistent")
