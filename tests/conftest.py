import os
import sys

import pytest
import torch

# variant tests switch measured alternatives with their DV_* A/B variables, which the package honours
# only in ablation mode (deconv_api_amd/knobs.py); set before any package module reads its switches
os.environ.setdefault("DV_ABLATIONS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    has_gpu = torch.cuda.is_available()
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords and not has_gpu:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native_lib():
    """The HIP extension; on a GPU box a missing build is a hard failure, never a skip."""
    from deconv_api_amd.ops import native

    return native.load(build_if_missing=True)


@pytest.fixture(scope="session")
def small_specs():
    from deconv_api_amd.models.vgg16 import vgg16_specs

    return vgg16_specs(width_div=8, image_size=32, fc=64, classes=10)
