import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ORACLE_DIR = os.path.join(ROOT, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def fgo():
    import fgo as m  # oracle/fgo.py — test infrastructure
    m.lib()
    return m


@pytest.fixture(scope="session")
def pkg():
    import _pkg
    return _pkg.load()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True


@pytest.fixture(scope="session")
def variants(pkg, gpu_available):
    """The measurement variants (fused waves, probe summary) are in libfgi_variants.so only
    (make -C stl.fusion_amd/csrc variant-all; FGI_LIBRARY selects it): skip their tests otherwise."""
    g = pkg.Graph(64)
    try:
        g.set_option(pkg.fgi.OPT_FUSED, 0)
        try:
            g.set_option(pkg.fgi.OPT_FUSED, 1)
        except pkg.FgiError as e:
            if e.status == pkg.fgi.ENOTSUP:
                pytest.skip("measurement variant: run with FGI_LIBRARY=stl.fusion_amd/lib/libfgi_variants.so")
            raise
    finally:
        g.close()
    return True
