import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "audio-to-sheet-music_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def state_dict():
    from athd.weights import synthetic_state_dict
    return synthetic_state_dict(seed=0)


@pytest.fixture(scope="session")
def text_table():
    from athd.weights import synthetic_text_table
    return synthetic_text_table(4, seed=7)


@pytest.fixture(scope="session")
def oracle_model(state_dict):
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    return AudioTextHTDemucsRef(state_dict)
