"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "whisper.rs_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: full-size (1500-frame) parity cases")


@pytest.fixture(scope="session")
def model_cache(tmp_path_factory):
    d = os.environ.get("WMI_MODEL_CACHE") or str(tmp_path_factory.mktemp("models"))
    os.makedirs(d, exist_ok=True)
    os.environ["WMI_MODEL_CACHE"] = d
    return d


@pytest.fixture(scope="session")
def micro_model(model_cache):
    import synth
    return synth.model_path("micro", model_cache)


@pytest.fixture(scope="session")
def oracle_micro(micro_model):
    import pyoracle
    return pyoracle.OracleModel(micro_model)


def threads():
    return min(16, os.cpu_count() or 8)
