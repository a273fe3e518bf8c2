"""Build libdecds_rlnc.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

The .so is git-ignored but travels to the GPU box with the gpurun snapshot; nothing is JIT-built
at import time, so a missing library fails loudly in decds_amd._capi.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdecds_rlnc.so")
# measurement only (bench.py's pattern ceilings): the same sources with DECDS_STUDY_PATTERN, i.e. the
# streaming kernels' memory pattern without their lookups (wrong bytes by design, never the product)
PATTERN_LIB = os.path.join(HERE, "..", "tools", "bin", "libdecds_pattern.so")
SOURCES = ["rlnc_kernels.hip", "commit_kernels.hip", "capi.cpp", "host_util.cpp", "host_mem.cpp", "chunkset.cpp", "blob.cpp",
           "commit.cpp", "wire.cpp", "blake3_host.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# backend options of the shipped build: the register-pressure trackers' schedules measured −0.4 %
# encode / −0.25 % decode / −0.2…−0.5 % fused ChunkSet::new on two boxes (r05u, r05v)
MLLVM = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
         "-Wno-unused-command-line-argument", "-I" + os.path.join(HERE, "..", "include")]


def _stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "decds_rlnc.h"),
                                                                 os.path.abspath(__file__)]  # flags live here
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, defines=(), out=None, mllvm=()):
    """Compile the library; `defines` (e.g. ["DECDS_WG=512"]), `mllvm` (LLVM backend options) and
    `out` build a tuning variant."""
    lib = out or LIB
    if not force and out is None and not _stale():
        return LIB
    tag = "_".join([d.replace("=", "_") for d in defines] + [m.strip("-").replace("=", "") for m in mllvm]) or "default"
    objdir = os.path.join(HERE, "..", "build", "obj", tag)
    os.makedirs(objdir, exist_ok=True)
    objs, procs = [], []
    for s in SOURCES:
        o = os.path.join(objdir, s + ".o")
        objs.append(o)
        cmd = [HIPCC] + FLAGS + MLLVM + ["-D" + d for d in defines] + [x for m in mllvm for x in ("-mllvm", m)] + \
              ["-c", os.path.join(CSRC, s), "-o", o]
        if s.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), out.decode()))
        if verbose and out.strip():
            sys.stderr.write(out.decode())
    tmp = lib + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stdout.decode()))
    os.replace(tmp, lib)
    return lib


def build_pattern(force=False, verbose=True):
    """tools/bin/libdecds_pattern.so: the pattern-ceiling build bench.py loads beside the product"""
    if not force and not _stale(PATTERN_LIB):
        return PATTERN_LIB
    os.makedirs(os.path.dirname(PATTERN_LIB), exist_ok=True)
    # decds=decds_pattern: every C++ symbol of this build, kernels included, lives in namespace
    # decds_pattern (the token `decds` appears in the sources only as that namespace's name), so a
    # rocprof trace of a process that loads both libraries lists the pattern launches under their own
    # names (_ZN13decds_pattern...) and never merges them into the product kernels' statistics
    return build(force=True, verbose=verbose, defines=["DECDS_STUDY_PATTERN=1", "decds=decds_pattern"], out=PATTERN_LIB)


COPYPATTERN_LIB = os.path.join(HERE, "..", "tools", "bin", "libdecds_copypattern.so")
COPYPATTERN_SRC = os.path.join(HERE, "..", "tools", "copypattern.hip")


def build_copypattern(force=False):
    """tools/bin/libdecds_copypattern.so: the decode's copy ceiling bench.py times (measurement only)"""
    if not force and os.path.exists(COPYPATTERN_LIB) and \
            os.path.getmtime(COPYPATTERN_LIB) >= max(os.path.getmtime(COPYPATTERN_SRC),
                                                     os.path.getmtime(os.path.join(CSRC, "rlnc_layout.h"))):
        return COPYPATTERN_LIB
    os.makedirs(os.path.dirname(COPYPATTERN_LIB), exist_ok=True)
    tmp = COPYPATTERN_LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + CSRC, COPYPATTERN_SRC, "-o", tmp]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), r.stdout.decode()))
    os.replace(tmp, COPYPATTERN_LIB)
    return COPYPATTERN_LIB


if __name__ == "__main__":
    # python -m decds_amd.build [--force] [--variant NAME -DX=1 ... --mllvm=-opt=v ...]
    args = sys.argv[1:]
    defs = [a[2:] for a in args if a.startswith("-D")]
    mll = [a[len("--mllvm="):] for a in args if a.startswith("--mllvm=")]
    if "--variant" in args:
        name = args[args.index("--variant") + 1]
        vdir = os.path.join(HERE, "..", "build", "variants")
        os.makedirs(vdir, exist_ok=True)
        print(build(force=True, defines=defs, out=os.path.join(vdir, "lib_%s.so" % name), mllvm=mll))
    elif "--pattern" in args:
        print(build_pattern(force="--force" in args))
    else:
        print(build(force="--force" in args, defines=defs))
