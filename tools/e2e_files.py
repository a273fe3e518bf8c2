"""File-to-file rate of decds-bin's break / repair flow over the device path:
write a random blob, `break` it into metadata.commit + chunkset.N/shareXX.data, delete 5 random
shares per chunkset, `repair` it, compare, and print one JSON line with per-phase times.
usage: python tools/e2e_files.py [--gib 1] [--dir /dev/shm] [--batch 64]"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--dir", default="/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir())
    ap.add_argument("--batch", type=int, default=0, help="chunksets per device batch (0: the flow's default)")
    ap.add_argument("--module", default="files", help="decds_amd module holding the flow (A/B of versions)")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (torch's HIP runtime must initialise before the library creates its context)
    import decds_amd
    import importlib
    from decds_amd import codec
    files = importlib.import_module("decds_amd." + a.module)
    kw = {"batch": a.batch} if a.batch else {}
    from decds_amd._capi import N
    ctx = decds_amd.Context(0)
    size = int(a.gib * (1 << 30))
    work = tempfile.mkdtemp(prefix="decds_e2e_", dir=a.dir)
    try:
        blob = codec.fill_random_host(0xF11E5, size)
        src = os.path.join(work, "blob.data")
        blob.tofile(src)
        tb = {}
        t0 = time.perf_counter()
        header = files.break_blob(ctx, src, os.path.join(work, "shares"), timings=tb, **kw)
        t_break = time.perf_counter() - t0
        rng = np.random.default_rng(6)
        for c in range(header.get_num_chunksets()):
            for j in rng.permutation(N)[:5]:
                os.remove(os.path.join(work, "shares", "chunkset.%d" % c, "share%02d.data" % j))
        tr = {}
        t0 = time.perf_counter()
        out = files.repair_blob(ctx, os.path.join(work, "shares"), os.path.join(work, "repaired"), timings=tr,
                                **kw)
        t_repair = time.perf_counter() - t0
        same = bool(np.array_equal(np.fromfile(out, dtype=np.uint8), blob))
        gib = size / (1 << 30)
        print(json.dumps({"blob_GiB": gib, "chunksets": header.get_num_chunksets(), "batch": a.batch or "default", "module": a.module,
                          "workdir_fs": a.dir, "break_s": round(t_break, 3), "break_GiBps": round(gib / t_break, 3),
                          "break_phases_s": {k: round(v, 3) for k, v in tb.items()},
                          "repair_s": round(t_repair, 3), "repair_GiBps": round(gib / t_repair, 3),
                          "repair_phases_s": {k: round(v, 3) for k, v in tr.items()},
                          "shares_kept_per_chunkset": N - 5, "roundtrip_ok": same}), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
