import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "roce-test_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session")
def ctx():
    import roce_icrc

    c = roce_icrc.Context(1)
    yield c
    c.close()


@pytest.fixture
def ctx_env(monkeypatch):
    """Factory: a fresh one-GPU Context created under the given RICRC_*
    environment knobs (libroceicrc reads them once, in ricrc_create), e.g.
    ``ctx_env(RICRC_SCK_GRID=1)``."""
    import roce_icrc

    made = []

    def make(**env):
        for k, v in env.items():
            monkeypatch.setenv(k, str(v))
        try:
            c = roce_icrc.Context(1)
        finally:
            for k in env:
                monkeypatch.delenv(k)
        made.append(c)
        return c

    yield make
    for c in made:
        c.close()
