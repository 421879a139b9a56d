import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import sod_pkg  # noqa: E402

sod_pkg.load()

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libsod.so")


def golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def _ctx_session():
    from sift_based_od_amd import _lib
    c = _lib.Context(0)
    yield c
    c.close()


@pytest.fixture
def ctx(_ctx_session):
    _ctx_session.set_impl("i8")
    _ctx_session.set_match_kernel("auto")
    opts = {k: _ctx_session.get_option(k) for k in _ctx_session.OPTIONS}
    yield _ctx_session
    for k, v in opts.items():          # a test's set_option stays in that test
        _ctx_session.set_option(k, v)


@pytest.fixture(params=["auto", "fallback"])
def trig(request, ctx):
    """The device-trig parity mode (sod option trig_exact): "auto" = the probe's answer (on a
    glibc-2.35 FMA host the device cos / sin are the host's and nothing is redone);
    "fallback" = forced off, so the boundary guard (hough.hip sod_guard_resolve) and the host
    exact-means redo (sod_exact_xy_means) run as on a host whose libm differs.  The ctx
    fixture restores the option afterwards."""
    ctx.set_option("trig_exact", -1 if request.param == "auto" else 0)
    if request.param == "fallback":
        assert not ctx.trig_exact()
    return request.param
