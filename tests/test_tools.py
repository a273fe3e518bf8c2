"""CPU: every HIP microbenchmark under tools/ still compiles against the current sources (front end
and semantic checks for gfx950, no code generation), so the studies DESIGN.md cites stay runnable."""
import concurrent.futures
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def test_tool_microbenchmarks_compile():
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not in this image")
    srcs = sorted(glob.glob(os.path.join(ROOT, "tools", "*.hip")))
    assert len(srcs) >= 8, srcs

    def check(src):
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(ROOT, "decds_amd", "csrc"),
                            "-fsyntax-only", src], capture_output=True, text=True, timeout=300)
        return src, r.returncode, r.stderr[-1500:]

    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        bad = [(os.path.basename(s), err) for s, rc, err in ex.map(check, srcs) if rc != 0]
    assert not bad, bad


def test_study_builds_of_the_kernels_compile():
    # the timing-study forms profiles/HISTORY.md §8 cites (per-workgroup phase trace, no edge pass, the pattern
    # ceiling, the aligned-piece layouts) stay buildable
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not in this image")
    src = os.path.join(ROOT, "decds_amd", "csrc", "rlnc_kernels.hip")
    for defs in (["-DDECDS_PHASE_TRACE=1"], ["-DDECDS_PHASE_TRACE=1", "-DDECDS_STUDY_NO_EDGE=1"],
                 ["-DDECDS_STUDY_PATTERN=1"], ["-DDECDS_STUDY_ALIGNED_PIECES=1"], ["-DDECDS_STUDY_ALIGNED_PIECES=3"],
                 ["-DDECDS_STUDY_PLAN=1"], ["-DDECDS_STUDY_PLAN=2"], ["-DDECDS_PLAN_FAST=0"]):
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                            "-fsyntax-only"] + defs + [src], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (defs, r.stderr[-1500:])
