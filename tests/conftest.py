import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs the HIP kernels")
    config.addinivalue_line("markers", "perf: a wall-clock gate (kernel fractions of the HBM roofline, host-path "
                                       "rates); also marked gpu, deselect with -m 'gpu and not perf'")


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "rlnc_kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ctx():
    import decds_amd
    return decds_amd.Context(0)


@pytest.fixture(autouse=True)
def _device_status_after_gpu_test(request):
    """After every -m gpu test: wait for the device and fail THIS test if it left a device fault
    (a sticky error would otherwise surface in whichever later test syncs first, GPUTEST_r01)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    from decds_amd._capi import check, lib
    torch.cuda.synchronize()
    check(lib().decds_device_status(request.getfixturevalue("ctx").handle))


def _tuning(name, value):
    from decds_amd._capi import lib
    return lib().decds_tuning(name.encode(), value, 1)


@pytest.fixture(params=["tiles", "tiles8", "sweep"])
def decode_form(request):
    """Run a decoding test through every decode kernel form whatever its batch size: one-tile workgroups
    (rlnc_decode_kernel) with 16-column or 8-column lane blocks, and the persistent sweep
    (rlnc_decode_sweep_kernel), by the process-wide thresholds DECDS_DEC_SWEEP_MIN_N and
    DECDS_DEC_NARROW_MAX_N (decds_tuning; back to their start values afterwards)."""
    _tuning("DECDS_DEC_SWEEP_MIN_N", 1 if request.param == "sweep" else 1 << 62)
    _tuning("DECDS_DEC_NARROW_MAX_N", 1 << 62 if request.param == "tiles8" else 0)
    yield request.param
    _tuning("DECDS_DEC_SWEEP_MIN_N", (1 << 64) - 1)
    _tuning("DECDS_DEC_NARROW_MAX_N", (1 << 64) - 1)


@pytest.fixture(params=["cols16", "cols16_nt", "cols8"])
def encode_form(request):
    """Run an encoding test through every instantiation of the encode sweep whatever its batch size:
    16-column lane blocks (batches above DECDS_ENC_SMALL_MAX_N) with write-through (below
    DECDS_ENC_NT_MIN_N) or non-temporal coded-row stores, and the small-batch form's 8-column blocks."""
    _tuning("DECDS_ENC_SMALL_MAX_N", 1 << 62 if request.param == "cols8" else 0)
    _tuning("DECDS_ENC_NT_MIN_N", 0 if request.param == "cols16_nt" else 1 << 62)
    yield request.param
    _tuning("DECDS_ENC_SMALL_MAX_N", (1 << 64) - 1)
    _tuning("DECDS_ENC_NT_MIN_N", (1 << 64) - 1)
