"""The README's results table, generated from the bench lines under profiles/ (one
table from the recorded runs instead of hand-edited ranges). Reads every profiles/*_bench.json given
(default: the final runs listed in FINAL), prints a markdown table, and with --write replaces the block
between the README's `<!-- results:begin -->` / `<!-- results:end -->` markers.

usage: python tools/results_table.py [--write] [files ...]"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FINAL = ["r08zf_bench.json", "r09*_bench.json"]  # round 5's final library, round 6's runs
BEGIN, END = "<!-- results:begin -->", "<!-- results:end -->"


def load(path):
    with open(path) as f:
        lines = [ln for ln in f if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def fmt(x, nd=3):
    return "—" if x is None else ("%.*f" % (nd, x))


def row(tag, d):
    rf = d["roofline"]
    enc, dec = rf["encode"], rf["decode"]
    sweep = {x["chunksets"]: x for x in (d.get("encode_batch_sweep") or [])}
    cb = d.get("cpu_baseline") or {}
    e2e = d.get("end_to_end") or {}
    api = {x["blob_bytes"]: x for x in ((d.get("api_shapes") or {}).get("sizes") or [])}
    g1 = api.get(1 << 30, {})
    return "| %s | **%.2f** | %s | %s | %s | %s | %s | %s / %s | %s | %s |" % (
        tag, d["value"], fmt(enc["frac"]), fmt(dec["frac"]), fmt(dec.get("frac_of_copy_pattern")),
        fmt((sweep.get(1) or {}).get("frac")), fmt((sweep.get(16) or {}).get("frac")),
        fmt(e2e.get("encode_blob_GiBps"), 1), fmt(e2e.get("repair_blob_GiBps"), 1),
        fmt((g1.get("blob_new") or {}).get("warm_GiBps"), 1),
        "%s (%s CPUs)" % (fmt(cb.get("value"), 1), cb.get("cores")) if cb else "—")


def table(files):
    out = ["| run | GiB/s (cfg3) | encode frac | decode frac | decode / its copy ceiling | encode frac at 1 cs | at 16 cs "
           "| end-to-end encode / repair GiB/s (1 GiB) | Blob::new warm GiB/s (1 GiB) | CPU baseline GiB/s |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for p in files:
        d = load(p)
        if d and d.get("roofline"):
            out.append(row(os.path.basename(p).replace("_bench.json", ""), d))
    return "\n".join(out)


def main():
    args = [a for a in sys.argv[1:] if a != "--write"]
    files = args or sorted({p for pat in FINAL for p in glob.glob(os.path.join(ROOT, "profiles", pat))})
    t = table(files)
    print(t)
    if "--write" in sys.argv:
        path = os.path.join(ROOT, "README.md")
        with open(path) as f:
            s = f.read()
        i, j = s.index(BEGIN) + len(BEGIN), s.index(END)
        with open(path, "w") as f:
            f.write(s[:i] + "\n" + t + "\n" + s[j:])


if __name__ == "__main__":
    main()
