"""CPU-side tests of the C-ABI library: it loads, exports every symbol include/decds_rlnc.h
declares, and its host-only control-path helpers agree with the oracle. No compute call is made
here (no GPU in this container); without a device every compute entry point must refuse loudly."""
import ctypes
import os
import re

import numpy as np
import pytest

import decds_amd
from decds_amd import _capi
import oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "decds_rlnc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(decds_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _capi.lib()
    declared = header_functions()
    assert len(declared) >= 20
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(_capi.EXPORTED) == declared


def test_status_codes_match_header():
    src = open(os.path.join(ROOT, "include", "decds_rlnc.h")).read()
    codes = {int(v.strip("()")) for v in re.findall(r"#define DECDS_(?:OK|ERR_[A-Z_]+)\s+(\(?-?\d+\)?)", src)}
    assert codes == set(_capi.STATUS_NAMES)
    lib = _capi.lib()
    for code in _capi.STATUS_NAMES:
        assert lib.decds_status_string(code) not in (None, b"unknown status")


def test_no_device_refuses_loudly():
    lib = _capi.lib()
    if lib.decds_device_count() > 0:
        pytest.skip("a device is visible")
    h = ctypes.c_void_p()
    assert lib.decds_ctx_create(0, ctypes.byref(h)) == _capi.STATUS["NoDevice"]
    assert b"device" in lib.decds_last_error()
    with pytest.raises(decds_amd.DecdsError) as e:
        decds_amd.Context(0)
    assert e.value.kind == "NoDevice"
    # a null context is refused by every batch entry point
    assert lib.decds_encode_batch(None, None, 1, None, None, _capi.CODED_PIECE_BYTES, None) == _capi.STATUS["InvalidArgument"]


def test_chunkset_new_invalid_size_before_device():
    # chunkset.rs:285-298 — the size check precedes any device work
    lib = _capi.lib()
    h = ctypes.c_void_p()
    for n in (_capi.CHUNKSET_BYTES - 1, _capi.CHUNKSET_BYTES + 1):
        buf = bytes(n)
        assert lib.decds_chunkset_new(None, 0, buf, n, None, ctypes.byref(h)) == _capi.STATUS["InvalidChunksetSize"]
        assert str(n) in lib.decds_last_error().decode()


def test_fill_random_host_matches_oracle():
    for seed, off, n in [(1, 0, 100), (0xDEC05001, 12345, 4097), (7, 3, 17)]:
        a = decds_amd.codec.fill_random_host(seed, n, off) if hasattr(decds_amd, "codec") else None
        from decds_amd import codec
        a = codec.fill_random_host(seed, n, off)
        assert np.array_equal(a, o.fill_random(seed, n, off))


def test_rank_push_matches_oracle():
    lib = _capi.lib()
    rng = np.random.default_rng(11)
    for _ in range(300):
        b1, p1, r1 = np.zeros(100, np.uint8), np.zeros(10, np.uint8), ctypes.c_uint32(0)
        b2, p2, r2 = np.zeros(100, np.uint8), np.zeros(10, np.uint8), ctypes.c_size_t(0)
        for _ in range(13):
            cv = (rng.integers(0, 4, 10) * rng.integers(0, 2, 10)).astype(np.uint8)
            u1 = lib.decds_rank_push(b1.ctypes.data, p1.ctypes.data, ctypes.byref(r1), cv.ctypes.data, 0x11D)
            u2 = o.lib().orc_rank_push(o._p(b2), o._p(p2), ctypes.byref(r2), o._p(cv), 10, 0x11D)
            assert u1 == u2
        assert r1.value == r2.value
        assert np.array_equal(b1[: 10 * r1.value], b2[: 10 * r2.value])


def test_layout_constants():
    assert _capi.PIECE_BYTES == o.L == 1048577
    assert _capi.CODED_PIECE_BYTES == o.F
    assert _capi.CHUNKSET_BYTES == o.CS


def test_decode_kernel_by_batch_size():
    # launch_decode (rlnc_kernels.hip decode_sweeps): the persistent sweep from 1536 chunksets on,
    # one-tile workgroups below; decds_tuning moves the threshold for the process (UINT64_MAX = back
    # to the start value); the environment variable of the same name sets that start value, read once
    import subprocess
    import sys
    lib = _capi.lib()
    name = lambda n: lib.decds_decode_kernel_name(n).decode()  # noqa: E731
    tune = lambda k, v, s=1: lib.decds_tuning(k.encode(), v, s)  # noqa: E731
    reset = (1 << 64) - 1
    try:
        if "DECDS_DEC_SWEEP_MIN_N" not in os.environ:
            assert tune("DECDS_DEC_SWEEP_MIN_N", reset) == 1536
            assert name(1) == name(255) == name(1535) == "rlnc_decode_kernel"
            assert name(1536) == name(1639) == "rlnc_decode_sweep_kernel"
        assert tune("DEC_SWEEP_MIN_N", 1) == 1 and name(1) == "rlnc_decode_sweep_kernel"  # prefix optional
        tune("DECDS_DEC_SWEEP_MIN_N", 1 << 40)
        assert name(1639) == "rlnc_decode_kernel"
        assert tune("DECDS_DEC_SWEEP_MIN_N", 0, 0) == 1 << 40  # read only
        if "DECDS_ENC_SMALL_MAX_N" not in os.environ:
            assert tune("DECDS_ENC_SMALL_MAX_N", 0, 0) == 2
        if "DECDS_ENC_NT_MIN_N" not in os.environ:
            assert tune("DECDS_ENC_NT_MIN_N", 0, 0) == 256
        for knob, default in (("DECDS_PLAN_DECODE_MAX_N", 2), ("DECDS_DEC_NARROW_MAX_N", 2)):
            if knob not in os.environ:
                assert tune(knob, 0, 0) == default, knob
        assert tune("ENC_NT_MIN_N", 5) == 5 and tune("DECDS_ENC_NT_MIN_N", reset) != 5
        assert tune("NO_SUCH_KNOB", 5) == reset
    finally:
        tune("DECDS_DEC_SWEEP_MIN_N", reset)
        tune("DECDS_ENC_SMALL_MAX_N", reset)
    code = ("import sys; sys.path.insert(0, %r); from decds_amd import _capi; L = _capi.lib(); "
            "n = lambda k: L.decds_decode_kernel_name(k).decode(); "
            "assert n(6) == 'rlnc_decode_kernel' and n(7) == 'rlnc_decode_sweep_kernel'; "
            "assert L.decds_tuning(b'DECDS_DEC_SWEEP_MIN_N', (1 << 64) - 1, 1) == 7" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, DECDS_DEC_SWEEP_MIN_N="7"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]


def test_library_consumes_its_hip_failures():
    # hip_status.h: hip_launch_begin treats an error pending on the thread as left by a HIP call
    # outside the library, so the library must consume every failure of its own calls (decds_hip_error,
    # hip_tolerate or an explicit hipGetLastError). Flags: a HIP call cast to (void) or called as a bare
    # statement (its status dropped, possibly left pending), and a (void)-cast drain() of a stream set.
    import re
    csrc = os.path.join(ROOT, "decds_amd", "csrc")
    bad = []
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".cpp", ".hip", ".h")):
            continue
        with open(os.path.join(csrc, f)) as fh:
            for no, line in enumerate(fh, 1):
                code = line.split("//")[0]
                if re.search(r"\(void\)\s*(hip(?!GetLastError)\w+|\w*drain)\s*\(", code):
                    bad.append("%s:%d: %s" % (f, no, line.strip()))
                if re.match(r"^\s*hip(?!LaunchKernelGGL|GetLastError)[A-Z]\w*\(", code):
                    bad.append("%s:%d: %s" % (f, no, line.strip()))
    assert not bad, "\n".join(bad)


def _hip_versions(path, section):
    """hip_X.Y symbol versions a shared object needs ("needs") or defines ("defs"), from readelf -V"""
    import subprocess
    out = subprocess.run(["readelf", "-V", path], capture_output=True, text=True, check=True).stdout
    if section == "needs":
        out = out.split("Version needs", 1)[-1]
        return set(re.findall(r"Name: (hip_[0-9.]+)\s+Flags", out))
    out = out.split("Version definition", 1)[-1].split("Version needs", 1)[0]
    return set(re.findall(r"Name: (hip_[0-9.]+)", out))


@pytest.mark.parametrize("lib", ["decds_amd/libdecds_rlnc.so", "tools/bin/libdecds_pattern.so"])
def test_library_needs_only_hip_versions_torch_provides(lib):
    # The library is loaded into processes whose HIP runtime is torch's bundled libamdhip64 (ROCm 7.0
    # here), not /opt/rocm's (7.2): a HIP call newer than that runtime (hipMemcpyBatchAsync needs
    # hip_7.1) makes the library fail to load at all there. Every hip_X.Y version it needs must be one
    # torch's runtime defines.
    import shutil
    torch = pytest.importorskip("torch")
    if not shutil.which("readelf"):
        pytest.skip("readelf not in this image")
    path = os.path.join(ROOT, lib)
    if not os.path.exists(path):
        pytest.skip("%s not built" % lib)
    rt = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if not os.path.exists(rt):
        pytest.skip("torch has no bundled HIP runtime")
    needs, defs = _hip_versions(path, "needs"), _hip_versions(rt, "defs")
    assert needs, "no hip_* version needs found in %s" % lib
    assert needs <= defs, sorted(needs - defs)
