#!/bin/bash
# One parametrised GPU-box session for tuning work (replaces round 1-3's one-off tools/sessions/*.sh,
# in git history up to 506a811). Steps run in the order given; every step has its own time limit and
# the first failure ends the session (no GPU step after a failed one).
#
# usage: bash tools/ab_session.sh OUTDIR STEP [STEP ...]
#   parity:LIB          GPU test suite against a variant build (DECDS_LIB=LIB; LIB=default: the in-tree one)
#   ab:N1,N2:LIB_A,LIB_B[,...]      tools/abbench.py --check (encode / plan / decode, in-process A/B) per N
#   fuse:N1,N2:LIB_A,LIB_B[,...]    tools/fusebench.py (fused ChunkSet::new) per N
#                                   a LIB may be "default" (the in-tree build) and carry "@KNOB=V" (a decds_tuning
#                                   launch-shape knob set before each of its runs: default@DECDS_ENC_SMALL_MAX_N=64)
#   bench:CFG                       tools/gpu_session.sh (tests, smoke, bench, rocprofv3 trace + PMC) at CFG
#   run:CMD                         any command (e.g. run:tools/bin/ldsconf), output to OUTDIR/run.log
# Variant builds: python -m decds_amd.build --variant NAME -DX=1 ... -> build/variants/lib_NAME.so
set -o pipefail
out=${1:?outdir}; shift
mkdir -p "$out"
export TMPDIR=/tmp
# a line every minute under $out: the first `import torch` on a fresh box can take minutes without
# output, which the GPU service takes for a hang (every step still has its own time limit)
( while sleep 60; do date +%T >> "$out/heartbeat"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
fail() { echo "$1 FAILED"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}
  case $kind in
    parity)
      lib=$arg; log=$out/parity_$(basename "$lib" .so).log
      if [ "$lib" = default ]; then unset DECDS_LIB; else export DECDS_LIB=$lib; fi
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$log" 2>&1 || fail parity "$log"
      unset DECDS_LIB; tail -1 "$log" ;;
    ab|fuse)
      sizes=${arg%%:*}; libs=${arg#*:}; tool=tools/abbench.py; extra="--check"
      [ "$kind" = fuse ] && { tool=tools/fusebench.py; extra=""; }
      # every variant build passes the static ISA checks (no static LDS under the tables, no spills, the
      # tile counter's pending register read only after its wait) before it runs: a variant that
      # spilled that register hung a box's A/B (r06z14). (Not the guard presence checks — sweep
      # guard, LDS-base guard: their own cost A/Bs run builds without them.)
      for spec in ${libs//,/ }; do
        lib=${spec%%[:@]*}
        [ "$lib" = default ] && continue
        DECDS_LIB=$lib timeout -k 10 300 python -m pytest tests/test_isa.py -q -p no:cacheprovider -k "not trap and not lds_base" > "$out/isa_$(basename "$lib" .so).log" 2>&1 \
          || fail "isa check of $lib" "$out/isa_$(basename "$lib" .so).log"
      done
      for n in ${sizes//,/ }; do
        timeout -k 10 300 python -u $tool $extra --n "$n" --rounds 12 ${libs//,/ } >> "$out/$kind.jsonl" 2>> "$out/$kind.err" || fail "$kind n=$n" "$out/$kind.err"
      done
      cat "$out/$kind.jsonl" ;;
    bench)
      bash tools/gpu_session.sh "$out/session_$arg" 20 "$arg" || exit 1 ;;
    run)
      timeout -k 10 300 $arg >> "$out/run.log" 2>&1 || fail "run $arg" "$out/run.log"
      tail -20 "$out/run.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo ab-session-ok
