import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs the HIP path through the C ABI")
    config.addinivalue_line("markers", "slow: multi-second CPU oracle runs")


@pytest.fixture(scope="session")
def oracle_lib():
    from tests import oracle

    return oracle.load()


@pytest.fixture(scope="session")
def fpm_lib():
    from fastest_image_pattern_matching_amd import _lib

    return _lib.load()


@pytest.fixture(scope="session")
def templates():
    from fastest_image_pattern_matching_amd import synth

    return synth.load_templates()


@pytest.fixture(scope="session")
def gpu_matcher_factory():
    """Factory of GPU matchers; fails (does not skip) when the HIP library or device is unusable."""
    from fastest_image_pattern_matching_amd import TemplateMatcher

    def make(**params):
        m = TemplateMatcher(0)
        for k, v in params.items():
            setattr(m._params, k, v)
        return m

    return make
