"""Static checks on the built gfx950 code (CPU only: disassembles the library, runs nothing).

The persistent sweeps (rlnc_encode_sweep_kernel, rlnc_decode_sweep_kernel in
decds_amd/csrc/rlnc_kernels.hip) bump their tile counter with an inline-asm
`global_atomic_add ... sc0` whose returned value lands in a VGPR the compiler does not know is
still pending; the kernels wait for it themselves, a step later, with `s_waitcnt vmcnt(N)` (N = the
memory operations issued after it). That is only sound while the compiler neither reads nor copies
nor spills that VGPR before such a wait — a property of the generated code, so it is checked on the
generated code: for every returning atomic, on every control-flow path from it (branches followed,
both ways for conditional ones, loops until the counts repeat), the first instruction that names its
destination register must come after a vmcnt wait that covers the atomic (count <= memory
operations issued since). (A scan in program order was enough until the compiler placed a loop's
tail after its atomic: the scan then walked past an `s_branch` into the epilogue.)
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

VMEM = ("buffer_", "global_", "scratch_", "flat_")


LIBS = ("product", "pattern")  # the in-tree library, and bench.py's pattern-ceiling build (it runs on the GPU too)


def _lib(which="product"):
    from decds_amd import build

    if which == "pattern":
        return build.build_pattern(verbose=False)
    return os.environ.get("DECDS_LIB") or build.build(verbose=False)  # a variant build, or the in-tree one


def _device_code(tmp_path, which="product"):
    lib = _lib(which)
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
    """{symbol: [(byte address, instruction)]} of the disassembly."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None:
            parts = line.split("//")
            ins = parts[0].strip()
            am = re.match(r"\s*([0-9A-Fa-f]+):", parts[1]) if len(parts) > 1 else None
            if ins and not ins.endswith(":") and am:
                cur.append((int(am.group(1), 16), ins))
    return funcs


def _names_vgpr(ins, reg):
    for m in re.finditer(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]", ins):
        if m.group(1) is not None and int(m.group(1)) == reg:
            return True
        if m.group(2) is not None and int(m.group(2)) <= reg <= int(m.group(3)):
            return True
    return False


def _successors(fn, idx, at):
    """instruction indices that can follow fn[idx] (s_branch: its target; s_cbranch_*: both)."""
    addr, ins = fn[idx]
    op = ins.split()[0]
    if op in ("s_endpgm", "s_setpc_b64", "s_swappc_b64"):
        return []
    nxt = [idx + 1] if idx + 1 < len(fn) else []
    if op == "s_branch" or op.startswith("s_cbranch"):
        simm = int(ins.split()[1], 0) & 0xFFFF
        simm -= 0x10000 if simm & 0x8000 else 0
        tgt = at.get(addr + 4 + 4 * simm)
        tgts = [tgt] if tgt is not None else []
        return tgts if op == "s_branch" else nxt + tgts
    return nxt


def _unsafe_uses(fn):
    """(atomic index, offending instruction) for every returning atomic read too early on some path."""
    at = {a: i for i, (a, _) in enumerate(fn)}
    bad = []
    for i, (_, ins) in enumerate(fn):
        m = re.match(r"^global_atomic_add v(\d+), .*\bsc0\b", ins)
        if not m:
            continue
        reg = int(m.group(1))
        seen, stack = set(), [(j, 0) for j in _successors(fn, i, at)]
        while stack and not bad:
            j, issued = stack.pop()
            if (j, issued) in seen:
                continue
            seen.add((j, issued))
            nxt = fn[j][1]
            w = re.search(r"s_waitcnt\b.*\bvmcnt\((\d+)\)", nxt)
            if w and int(w.group(1)) <= issued:
                continue  # the atomic has landed on this path
            if _names_vgpr(nxt, reg) and not w:
                bad.append((i, nxt))
                break
            inc = 1 if nxt.split()[0].startswith(VMEM) else 0
            stack.extend((k, min(issued + inc, 64)) for k in _successors(fn, j, at))
    return bad


@pytest.mark.parametrize("which", LIBS)
def test_counter_atomics_are_waited_for_before_use(tmp_path, which):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    funcs = _functions(_device_code(tmp_path, which))
    sweeps = {k: v for k, v in funcs.items() if "sweep_kernel" in k}
    assert any("encode_sweep" in k for k in sweeps), sorted(funcs)[:20]
    checked = 0
    for name, ins in sweeps.items():
        checked += sum(1 for _, x in ins if re.match(r"^global_atomic_add v\d+, .*\bsc0\b", x))
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
    # control flow: an early read jumped over (s_branch) is not on the path; one on either side of a
    # conditional branch is
    jumped = ["global_atomic_add v7, v[0:1], v2, off sc0", "s_branch 1", "v_mov_b32_e32 v12, v7", "s_waitcnt vmcnt(0)",
              "v_mov_b32_e32 v12, v7", "s_endpgm"]
    either = ["global_atomic_add v7, v[0:1], v2, off sc0", "s_cbranch_scc1 1", "v_mov_b32_e32 v12, v7", "s_waitcnt vmcnt(0)",
              "s_endpgm"]
    def fn(xs):  # byte addresses: 8-byte memory instructions, 4-byte others (branch offsets count dwords)
        out, a = [], 0
        for x in xs:
            out.append((a, x))
            a += 8 if x.startswith(VMEM) else 4
        return out
    assert _unsafe_uses(fn(early)) and not _unsafe_uses(fn(late)) and _unsafe_uses(fn(ranged))
    assert not _unsafe_uses(fn(jumped)) and _unsafe_uses(fn(either))


def _kernel_notes(tmp_path, which="product"):
    """{kernel symbol: {metadata key: value}} from the gfx950 code objects' AMDGPU notes"""
    lib = _lib(which)
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


@pytest.mark.parametrize("which", LIBS)
def test_table_kernels_have_no_static_lds(tmp_path, which):
    # The streaming kernels' lookups are inline-asm ds_read_b128 with absolute LDS offsets: their
    # tables must start at LDS address 0, i.e. the dynamic area must come first. A static __shared__
    # variable in such a kernel is placed before the dynamic area and shifts every table (round 4's
    # first TailLds build did that: repaired bytes wrong). Their group segment must be 0.
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    notes = _kernel_notes(tmp_path, which)
    table = {k: v for k, v in notes.items()
             if any(s in k for s in ("encode_sweep_kernel", "decode_sweep_kernel", "rlnc_decode_kernel", "plan_decode_kernel",
                                     "encode_hash_kernel"))}
    assert len(table) >= 5, sorted(notes)
    for name, md in table.items():
        assert md.get("group_segment_fixed_size") == "0", (name, md.get("group_segment_fixed_size"))
        assert md.get("private_segment_fixed_size") == "0", (name, "spills to scratch")


@pytest.mark.parametrize("which", LIBS)
def test_sweeps_trap_instead_of_spinning(tmp_path, which):
    # every persistent sweep carries the guard (rlnc_kernels.hip sweep_guard): a next tile not past the
    # current one — a counter value read before its atomic landed, the round-4 3-wave hang (profiles/
    # HISTORY.md §8) — ends the kernel with s_trap instead of an endless loop over one tile
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    funcs = _functions(_device_code(tmp_path, which))
    sweeps = {k: v for k, v in funcs.items() if "sweep_kernel" in k}
    assert sum("encode_sweep" in k for k in sweeps) >= 5 and any("decode_sweep" in k for k in sweeps), sorted(sweeps)
    for name, ins in sweeps.items():
        assert any(x.startswith("s_trap 2") for _, x in ins), name


@pytest.mark.parametrize("which", LIBS)
def test_table_kernels_guard_their_lds_base(tmp_path, which):
    # rlnc_kernels.hip tables_at_lds_zero(): every kernel whose inline-asm lookups address the tables
    # from LDS byte 0 checks its static LDS size at entry and traps if it is not 0 (the compare survives
    # as `s_cmp_eq_u32 0, 0` or `s_cmp_lg_u32 0, 0` — the size is filled in after instruction selection)
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    funcs = _functions(_device_code(tmp_path, which))
    table = {k: v for k, v in funcs.items() if any(s in k for s in ("encode_sweep_kernel", "decode_sweep_kernel",
                                                                    "rlnc_decode_kernel", "encode_hash_kernel", "plan_decode_kernel"))}
    assert len(table) >= 5, sorted(funcs)[:20]
    for name, ins in table.items():
        assert any(x.startswith("s_trap 2") for _, x in ins), name
        assert any(re.match(r"s_cmp_(eq|lg)_u32 0, 0$", x) for _, x in ins[:8]), (name, ins[:8])


def test_pattern_build_symbols_are_disjoint_from_the_product(tmp_path):
    # bench.py loads tools/bin/libdecds_pattern.so (wrong bytes by design) into the same process as the
    # product: its kernels must carry names of their own (namespace decds_pattern, decds_amd/build.py
    # build_pattern), so no profile can merge their launches into the product kernels' statistics
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    (tmp_path / "p").mkdir()
    (tmp_path / "q").mkdir()
    prod, pat = set(_kernel_notes(tmp_path / "p", "product")), set(_kernel_notes(tmp_path / "q", "pattern"))
    assert len(prod) >= 10 and len(pat) >= 10, (len(prod), len(pat))
    assert not prod & pat, sorted(prod & pat)[:5]
    assert all(k.startswith("_ZN5decds") for k in prod), [k for k in prod if not k.startswith("_ZN5decds")][:5]
    assert all(k.startswith("_ZN13decds_pattern") for k in pat), [k for k in pat if not k.startswith("_ZN13decds_pattern")][:5]
    # the host-side launch stubs too
    nm = lambda lib: {ln.split()[-1] for ln in subprocess.run(["nm", lib], capture_output=True, text=True, check=True)
                      .stdout.splitlines() if "_kernel" in ln and ln.split()[-1].startswith("_ZN")}
    hp, hq = nm(_lib("product")), nm(_lib("pattern"))
    assert hp and hq and not hp & hq
