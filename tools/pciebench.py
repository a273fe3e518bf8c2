"""PCIe copy rates between page-locked host memory and HBM: H2D alone, D2H alone, and both at once
on two streams (full duplex?). Prints one JSON line. usage: python tools/pciebench.py --mib 1024"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    nb = a.mib << 20
    h_in = torch.empty(nb, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(nb, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(nb, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(nb, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run(h2d, d2h):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            if h2d:
                with torch.cuda.stream(s1):
                    d_in.copy_(h_in, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    h_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.reps

    run(True, True)
    th, td, tb = run(True, False), run(False, True), run(True, True)
    print(json.dumps({"MiB": a.mib, "h2d_GBps": round(nb / th / 1e9, 1), "d2h_GBps": round(nb / td / 1e9, 1),
                      "both_GBps_each": round(nb / tb / 1e9, 1), "both_GBps_total": round(2 * nb / tb / 1e9, 1)}))


if __name__ == "__main__":
    main()
