import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def engine():
    from genomealignmenttools_amd.gachain import Engine
    e = Engine(0)
    yield e
    e.close()


BLASTZ = [[91, -114, -31, -123], [-114, 100, -125, -31], [-31, -125, 100, -114],
          [-123, -31, -114, 91]]
