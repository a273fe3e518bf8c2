"""bench.py's JSON line on the device: the contract fields, and a roofline block that is internally
consistent — its `achieved` / `frac` belong to the kernel it names (the dominant one by time), and
match that kernel's own entry and the breakdown's GB/s."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_roofline_is_the_dominant_kernels():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--settle-s", "0.1",
                        "--no-cpu-baseline", "--no-commit", "--no-sweep"], capture_output=True, text=True, timeout=110,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    rf, bd = d["roofline"], d["breakdown"]
    enc, dec = rf["encode"], rf["decode"]
    dom = enc if bd["encode_ms"] >= bd["decode_ms"] else dec
    assert rf["kernel"] == dom["kernel"]
    assert rf["achieved"] == dom["achieved"] and rf["frac"] == dom["frac"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert enc["achieved"] == bd["encode_GBps"] and dec["achieved"] == bd["decode_GBps"]
    assert enc["kernel"].startswith("rlnc_encode")


@pytest.mark.gpu
def test_bench_rehearsal_runs_one_shard_of_a_larger_job():
    # --rehearse-shard R/W (the one-GPU run of cfg5's shards): rank 1 of a 2-GPU cfg2 job = chunksets
    # [103, 205) of a 2 GiB blob, the last one partial, every repaired chunkset checked inside bench.py
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--settle-s", "0.1",
                        "--no-cpu-baseline", "--no-commit", "--rehearse-shard", "1/2"], capture_output=True, text=True,
                       timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    reh = d["rehearsal"]
    assert reh["rank"] == 1 and reh["world"] == 2 and reh["first_chunkset"] == 103 and reh["chunksets"] == 102
    assert reh["shard_bytes"] == (2 << 30) - 103 * (10 << 20) and d["n_gpus"] == 1
    assert d["encode_batch_sweep"] is None and d["value"] > 0
