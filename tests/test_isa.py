"""Static checks on the built gfx950 code (CPU only: disassembles the library, runs nothing).

The persistent sweeps (rlnc_encode_sweep_kernel, rlnc_decode_sweep_kernel in
decds_amd/csrc/rlnc_kernels.hip) bump their tile counter with an inline-asm
`global_atomic_add ... sc0` whose returned value lands in a VGPR the compiler does not know is
still pending; the kernels wait for it themselves, a step later, with `s_waitcnt vmcnt(N)` (N = the
memory operations issued after it). That is only sound while the compiler neither reads nor copies
nor spills that VGPR before such a wait — a property of the generated code, so it is checked on the
generated code: for every returning atomic, scanning forward in program order, the first
instruction that names its destination register must come after a vmcnt wait that covers the
atomic (count <= memory operations issued since).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

VMEM = ("buffer_", "global_", "scratch_", "flat_")


def _device_code(tmp_path):
    from decds_amd import build

    lib = os.environ.get("DECDS_LIB") or build.build(verbose=False)  # a variant build, or the in-tree one
    work = tmp_path / "isa"
    work.mkdir()
    shutil.copy(lib, work / "lib.so")
    subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=work, check=True, capture_output=True)
    texts = []
    for f in sorted(os.listdir(work)):
        if "amdgcn" in f and "gfx950" in f:
            r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f], cwd=work, check=True, capture_output=True, text=True)
            texts.append(r.stdout)
    assert texts, "no gfx950 code object in the library"
    return "\n".join(texts)


def _functions(text):
    """{symbol: [instruction lines]} of the disassembly."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None:
            ins = line.split("//")[0].strip()
            if ins and not ins.endswith(":"):
                cur.append(ins)
    return funcs


def _names_vgpr(ins, reg):
    for m in re.finditer(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]", ins):
        if m.group(1) is not None and int(m.group(1)) == reg:
            return True
        if m.group(2) is not None and int(m.group(2)) <= reg <= int(m.group(3)):
            return True
    return False


def _unsafe_uses(ins_list):
    """(atomic index, offending instruction) for every returning atomic read too early."""
    bad = []
    for i, ins in enumerate(ins_list):
        m = re.match(r"^global_atomic_add v(\d+), .*\bsc0\b", ins)
        if not m:
            continue
        reg, issued = int(m.group(1)), 0
        for nxt in ins_list[i + 1:]:
            w = re.search(r"s_waitcnt\b.*\bvmcnt\((\d+)\)", nxt)
            if w and int(w.group(1)) <= issued:
                break  # the atomic has landed
            op = nxt.split()[0]
            if _names_vgpr(nxt, reg) and not w:
                bad.append((i, nxt))
                break
            if op.startswith(VMEM):
                issued += 1
            if op == "s_endpgm":
                break
    return bad


def test_counter_atomics_are_waited_for_before_use(tmp_path):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    funcs = _functions(_device_code(tmp_path))
    sweeps = {k: v for k, v in funcs.items() if "sweep_kernel" in k}
    assert any("encode_sweep" in k for k in sweeps), sorted(funcs)[:20]
    checked = 0
    for name, ins in sweeps.items():
        checked += sum(1 for x in ins if re.match(r"^global_atomic_add v\d+, .*\bsc0\b", x))
        assert not _unsafe_uses(ins), (name, _unsafe_uses(ins))
    assert checked >= 2


def test_checker_flags_an_early_read():
    # the checker itself: a copy of the returned register before any covering wait is flagged;
    # the same copy after vmcnt(1) with one load issued in between is not
    early = ["global_atomic_add v7, v[0:1], v2, off sc0", "buffer_load_dwordx4 v[8:11], v3, s[0:3], 0 offen",
             "v_mov_b32_e32 v12, v7", "s_waitcnt vmcnt(1)"]
    late = ["global_atomic_add v7, v[0:1], v2, off sc0", "buffer_load_dwordx4 v[8:11], v3, s[0:3], 0 offen",
            "s_waitcnt vmcnt(1)", "v_mov_b32_e32 v12, v7"]
    ranged = ["global_atomic_add v7, v[0:1], v2, off sc0", "scratch_store_dwordx2 off, v[6:7], off offset:4"]
    assert _unsafe_uses(early) and not _unsafe_uses(late) and _unsafe_uses(ranged)


def _kernel_notes(tmp_path):
    """{kernel symbol: {metadata key: value}} from the gfx950 code objects' AMDGPU notes"""
    from decds_amd import build

    lib = os.environ.get("DECDS_LIB") or build.build(verbose=False)
    work = tmp_path / "notes"
    work.mkdir()
    shutil.copy(lib, work / "lib.so")
    subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=work, check=True, capture_output=True)
    readelf = os.path.join(os.path.dirname(OBJDUMP), "llvm-readelf")
    kernels = {}
    for f in sorted(os.listdir(work)):
        if "amdgcn" not in f or "gfx950" not in f:
            continue
        r = subprocess.run([readelf, "--notes", f], cwd=work, check=True, capture_output=True, text=True)
        entry = None
        for line in r.stdout.splitlines():
            if re.match(r"^  - \.", line):  # a kernel entry of amdhsa.kernels starts (its keys sorted)
                entry = {}
            m = re.match(r"^  [- ] \.(\w+):\s+(\S+)", line)  # the entry's own keys, not its args'
            if entry is not None and m:
                entry[m.group(1)] = m.group(2)
                if m.group(1) == "name":
                    kernels[m.group(2)] = entry
    return kernels


def test_table_kernels_have_no_static_lds(tmp_path):
    # The streaming kernels' lookups are inline-asm ds_read_b128 with absolute LDS offsets: their
    # tables must start at LDS address 0, i.e. the dynamic area must come first. A static __shared__
    # variable in such a kernel is placed before the dynamic area and shifts every table (round 4's
    # first TailLds build did that: repaired bytes wrong). Their group segment must be 0.
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    notes = _kernel_notes(tmp_path)
    table = {k: v for k, v in notes.items()
             if any(s in k for s in ("encode_sweep_kernel", "decode_sweep_kernel", "rlnc_decode_kernel",
                                     "encode_hash_kernel"))}
    assert len(table) >= 5, sorted(notes)
    for name, md in table.items():
        assert md.get("group_segment_fixed_size") == "0", (name, md.get("group_segment_fixed_size"))
        assert md.get("private_segment_fixed_size") == "0", (name, "spills to scratch")
