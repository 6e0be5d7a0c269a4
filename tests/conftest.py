"""pytest configuration: the ``gpu`` marker selects tests that need an MI355X (run with -m gpu)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device); run with -m gpu')


@pytest.fixture(scope='session')
def od_golden():
    import numpy as np
    return np.load(os.path.join(GOLDEN, 'od_golden.npz'))


@pytest.fixture(scope='session')
def si_golden():
    import numpy as np
    return np.load(os.path.join(GOLDEN, 'si_golden.npz'))
