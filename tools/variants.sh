#!/bin/bash
# Time every built variant (build/variants/lib_*.so) with tools/kbench.py on the GPU box.
# usage (on the box): bash tools/variants.sh "103 1639" > gpurun_out/variants.jsonl
sizes=${1:-"103"}
for lib in build/variants/lib_*.so; do
  extra="--check"
  for n in $sizes; do
    DECDS_LIB=$lib timeout -k 10 120 python tools/kbench.py --n $n --reps 15 $extra --tag $(basename $lib .so) || exit 1
  done
done
