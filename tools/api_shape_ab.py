"""bench.py's api_shapes (the reference's build_blob / repair_blob benches through the blob API) at one
size, for A/B runs of library settings taken from the environment. One JSON line.

usage: DECDS_HOST_SPIN_US=0 python tools/api_shape_ab.py [--gib 1] [--tag spin0]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch  # noqa: F401  (device init as in bench.py)
    import decds_amd
    import bench
    ctx = decds_amd.Context(0)
    res = bench.api_shapes(ctx, sizes=[int(a.gib * (1 << 30))], repeats=5, repair_repeats=3)
    print(json.dumps({"tag": a.tag, "env": {k: v for k, v in os.environ.items() if k.startswith("DECDS_")}, "api_shapes": res}))


if __name__ == "__main__":
    main()
