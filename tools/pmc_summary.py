"""Summarise a tools/gpu_session.sh output directory into profiles/:
  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the bench command
  <tag>_pmc_summary.json   per-kernel mean of every PMC counter collected (separate passes)
  traffic.json             HBM bytes per launch of the codec kernels, read by bench.py:
                           (2 x FETCH_SIZE + WRITE_SIZE) x 1024 — FETCH_SIZE reads half the bytes of
                           wide streaming loads on gfx950 (MI355X_MICROARCH.md §HBM)
usage: python tools/pmc_summary.py gpurun_out/r01s1 r01 [config]"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(name):
    """'void decds::rlnc_encode_kernel<0>(...)' -> 'decds::rlnc_encode_kernel'"""
    return re.sub(r"<[^<>]*>$", "", re.sub(r"^void ", "", name.split("(")[0]))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    config = sys.argv[3] if len(sys.argv) > 3 else "cfg2"
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*_kernel_stats.csv"))[0]
    shutil.copy(stats, os.path.join(prof, "%s_kernel_stats.csv" % tag))
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(src, "pmc*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    summary = collections.defaultdict(dict)
    for (k, c), v in agg.items():
        if k.startswith("decds::"):
            summary[k][c] = sum(v) / len(v)
    durations = {kname(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(stats))}
    for k in summary:
        summary[k]["avg_duration_ns"] = durations.get(k)
    with open(os.path.join(prof, "%s_pmc_summary.json" % tag), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    traffic = {"config": config, "source": "profiles/%s_pmc_summary.json" % tag, "kernels": {}}
    for k, c in summary.items():
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            name = k.split("::")[-1]
            traffic["kernels"][name] = {"hbm_bytes_per_launch": round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024),
                                        "fetch_bytes_corrected": round(2 * c["FETCH_SIZE"] * 1024),
                                        "write_bytes": round(c["WRITE_SIZE"] * 1024)}
    # the bench line printed by the profiled run itself: its HIP-event averages are for the same
    # launches as the kernel trace
    tlog = os.path.join(src, "trace.log")
    if os.path.exists(tlog):
        for line in open(tlog):
            if line.startswith("{") and '"metric"' in line:
                with open(os.path.join(prof, "%s_bench_traced.json" % tag), "w") as f:
                    f.write(line)
    # the VALU issue roofline of the VALU-bound kernels (tools/isa_mix.py: SQ_INSTS_VALU x mean cycles per
    # VALU instruction of the built kernel's mix / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)), read by bench.py
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import isa_mix
        from decds_amd import build
        funcs = isa_mix.functions(isa_mix.disassemble(build.build(verbose=False)))
        for k, c in summary.items():
            name = k.split("::")[-1]
            sym = next((s for s in funcs if name in s), None)
            if sym and "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
                m = isa_mix.mix(funcs[sym])
                simd_cycles = isa_mix.SIMDS * c["GRBM_GUI_ACTIVE"] / isa_mix.XCDS
                traffic["kernels"].setdefault(name, {})["valu"] = {
                    "insts_per_launch": c["SQ_INSTS_VALU"], "cycles_per_valu": m["cycles_per_valu"],
                    "frac": round(c["SQ_INSTS_VALU"] * m["cycles_per_valu"] / simd_cycles, 4),
                    "frac_full_rate": round(c["SQ_INSTS_VALU"] * 2 / simd_cycles, 4)}
    except Exception as e:  # noqa: BLE001 - the traffic figures stand without it
        print("valu roofline skipped: %s" % e, file=sys.stderr)
    with open(os.path.join(prof, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
