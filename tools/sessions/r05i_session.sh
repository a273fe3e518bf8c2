#!/bin/bash
# FETCH_SIZE calibration for 8-byte-per-lane loads (MI355X_MICROARCH.md: only 16-B/lane streaming reads
# are calibrated, at exactly half): the sweep encode built with 8-column lane blocks (buffer_load_b64,
# every input byte read once) against the shipped 16-column build (b128) and the fused hash kernel (b64)
set -o pipefail
out=gpurun_out/r05i; mkdir -p $out
export TMPDIR=/tmp
for v in encdw2 base; do
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_$v -o run -- python3 tools/abbench.py --n 103 --rounds 2 --warmup-s 0.2 build/ab/lib_$v.so:1048704+16 > $out/pmc_$v.log 2>&1 || { echo PMC $v FAILED; tail -5 $out/pmc_$v.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fuse -o run -- python3 tools/fusebench.py --n 103 --rounds 2 --warmup-s 0.2 build/ab/lib_base.so > $out/pmc_fuse.log 2>&1 || { echo PMC fuse FAILED; tail -5 $out/pmc_fuse.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, re
for d in ("encdw2", "base", "fuse"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/r05i/pmc_%s/*counter_collection.csv" % d):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"^void ", "", r["Kernel_Name"].split("(")[0])
            agg[k].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "encode" in k or "hash" in k or "decode" in k or "digest" in k:
            print(d, k, "launches", len(v), "FETCH_SIZE KiB mean", round(sum(v) / len(v)), "bytes", round(sum(v) / len(v) * 1024))
PY
