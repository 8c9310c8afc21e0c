import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "spawns: starts GPU child processes; runs before anything touches the GPU here")


def pytest_sessionstart(session):
    # scenes/bun69k.cli is generated (deterministic, ~1.5 s) and not pushed to the GPU box
    from distraytracer_old_amd import scenes
    scenes.ensure_bun69k()


def pytest_collection_modifyitems(session, config, items):
    # child processes are started before this process initialises HIP (no exec / fork+exec
    # from a GPU-initialised process): the `spawns` tests go first, in their file order
    items.sort(key=lambda it: 0 if it.get_closest_marker("spawns") else 1)


@pytest.fixture(scope="session")
def gpu_available():
    from distraytracer_old_amd import rt
    return rt.device_count() > 0
