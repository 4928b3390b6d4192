import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libmec's HIP path)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_collection_modifyitems(config, items):
    pass


def pytest_collection_finish(session):
    # GPU runs: the tests' torch copies go through pinned memory
    # (tests/_pinned_copies.py)
    if any(item.get_closest_marker("gpu") for item in session.items):
        import torch
        if torch.cuda.is_available():
            import _pinned_copies
            _pinned_copies.install()


@pytest.fixture(scope="session")
def golden():
    import _oracle
    return _oracle.golden()


@pytest.fixture
def knobs():
    """Set libmec launch-shape knobs through mec_set_knob (the library reads
    the environment once; experiments change knobs through the API) and put
    every touched knob back to its built-in rule afterwards."""
    import memec_amd
    touched = set()

    def set_(name, value):
        touched.add(name)
        memec_amd.set_knob(name, value)
    yield set_
    for name in touched:
        memec_amd.set_knob(name, None)
