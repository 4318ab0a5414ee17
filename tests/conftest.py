import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950); run on the GPU box with -m gpu")
    config.addinivalue_line("markers", "slow: full BASELINE.json sizes")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle

    return Oracle()


@pytest.fixture(scope="session")
def kat():
    return json.loads((GOLDEN / "kat.json").read_text())["cases"]


@pytest.fixture(scope="session")
def batches():
    return json.loads((GOLDEN / "batches.json").read_text())


@pytest.fixture(scope="session")
def pattern_bytes():
    from tests.golden.make_golden import pattern_bytes as pb

    return pb
