"""VALU instruction mix of the built gfx950 kernels (static, from the disassembly) and the VALU
issue-roofline fraction of a profiled launch.

Why: the fused ChunkSet::new kernel (rlnc_encode_hash_kernel) is bound by vector issue, not HBM
(DESIGN.md §5.4). A wave64 VALU instruction occupies its SIMD-32 for 2 cycles at full rate
(v_xor_b32, v_add_u32, v_bitop3_b32, ...) and 4 cycles for the half-rate class measured on gfx950
(tools/valubench.hip, profiles/archive/r03a_valu_rates.jsonl: v_alignbit_b32, v_add3_u32, v_perm_b32, shifts,
SDWA forms, packed 16-bit adds). The issue roofline of a launch is then

    valu_frac = SQ_INSTS_VALU x c / (SIMDs x cycles),   cycles = GRBM_GUI_ACTIVE / 8 (XCDs),

with c the kernel's mean cycles per VALU instruction, weighted by its static mix (2 <= c <= 4).
It also counts, per BLAKE3 compression, the VALU instructions of the compression code against the
floor of 7 rounds x 8 G x 12 = 672 (commit_kernels.hip:9).

usage: python tools/isa_mix.py [pmc_summary.json]   (prints JSON)
"""
import collections
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
SIMDS = 1024  # 256 CUs x 4 SIMDs (MI355X)
XCDS = 8
HALF = re.compile(r"^v_(alignbit|alignbyte|add3|perm|lshlrev|lshrrev|ashrrev|lshl_or|lshl_add|and_or|or3|pk_|bfe|xad|"
                  r"mad_u32|mad_u64|mul_lo|mul_hi|cndmask_b32_e64)")
KERNELS = ("rlnc_encode_hash_kernel", "rlnc_encode_sweep_kernel", "rlnc_decode_sweep_kernel", "chunk_digest_kernel")


def disassemble(lib):
    work = tempfile.mkdtemp()
    try:
        shutil.copy(lib, os.path.join(work, "lib.so"))
        subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=work, check=True, capture_output=True)
        out = []
        for f in sorted(os.listdir(work)):
            if "amdgcn" in f and "gfx950" in f:
                out.append(subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f], cwd=work, check=True,
                                          capture_output=True, text=True).stdout)
        return "\n".join(out)
    finally:
        shutil.rmtree(work)


def functions(text):
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None:
            ins = line.split("//")[0].strip()
            if ins and not ins.endswith(":"):
                cur.append(ins.split()[0])
    return funcs


def mix(ops):
    valu = [o for o in ops if o.startswith("v_") and not o.startswith(("v_mfma", "v_readfirstlane", "v_readlane",
                                                                        "v_writelane"))]
    half = [o for o in valu if HALF.match(o) or "_sdwa" in o]
    c = collections.Counter(valu)
    return {"valu": len(valu), "half_rate": len(half), "full_rate": len(valu) - len(half),
            "cycles_per_valu": round((2 * (len(valu) - len(half)) + 4 * len(half)) / max(1, len(valu)), 3),
            "top": c.most_common(8)}


def main():
    from decds_amd import build
    lib = os.environ.get("DECDS_LIB") or build.build(verbose=False)
    funcs = functions(disassemble(lib))
    res = {"kernels": {}}
    for sym, ops in funcs.items():
        name = next((k for k in KERNELS if k in sym), None)
        if name:
            res["kernels"].setdefault(name, mix(ops))
    # the compression: chunk_digest_kernel is the compression plus a little staging, so its
    # v_alignbit count (4 rotates per G, 32 per round) gives the number of compressions inlined
    dg = funcs.get(next((s for s in funcs if "chunk_digest_kernel" in s), ""), [])
    n_align = sum(1 for o in dg if o.startswith("v_alignbit"))
    n_comp = max(1, round(n_align / 224))
    g_ops = [o for o in dg if re.match(r"^v_(alignbit|add3|xor|add_u32|bitop3|perm)", o)]
    res["compression"] = {"floor_valu": 672, "compressions_inlined_in_chunk_digest_kernel": n_comp,
                          "g_function_valu_per_compression": round(len(g_ops) / n_comp, 1)}
    if len(sys.argv) > 1:
        pmc = json.load(open(sys.argv[1]))
        for k, c in pmc.items():
            name = k.split("::")[-1]
            if name in res["kernels"] and "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
                m = res["kernels"][name]
                simd_cycles = SIMDS * c["GRBM_GUI_ACTIVE"] / XCDS
                m["pmc"] = {"SQ_INSTS_VALU": c["SQ_INSTS_VALU"], "GRBM_GUI_ACTIVE": c["GRBM_GUI_ACTIVE"],
                            "valu_frac_full_rate": round(c["SQ_INSTS_VALU"] * 2 / simd_cycles, 4),
                            "valu_frac": round(c["SQ_INSTS_VALU"] * m["cycles_per_valu"] / simd_cycles, 4),
                            "clock_GHz": round(c["GRBM_GUI_ACTIVE"] / XCDS / c["avg_duration_ns"], 3)
                            if c.get("avg_duration_ns") else None}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
