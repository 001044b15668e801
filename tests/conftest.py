import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The library reads its GM_* A/B knobs only with this opt-in (gm_internal.h
# knob(); the default build's list: include/emqx_gpu_match.h).  The suite sets
# knobs per test (monkeypatch) to cover every layout and walk form, so it opts
# in once here; with no knob set the library runs its defaults, as shipped.
# tests/test_host_cpu.py::test_knobs_need_the_ab_opt_in checks the gate itself.
os.environ.setdefault("EMQX_GM_AB", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def orc():
    """The CPU oracle (test infrastructure; built by `make -C oracle`)."""
    import subprocess
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    src = os.path.join(ROOT, "oracle", "emqx_oracle.cpp")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from oracle import oracle
    return oracle


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "suite_vectors.json")) as f:
        return json.load(f)
