#!/bin/bash
# bootstrap A/B: tools/boot_prof.py (768 chains) alternating two libraries, <reps> times each:
# boot_ab.sh <tag> <reps> <lib A> <lib B>
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out; tag=$1; reps=$2; A=$3; B=$4
mkdir -p $O; out=$O/${tag}_boot_ab.txt; : > $out
for i in $(seq $reps); do
  for L in $A $B; do
    VO_HIP_LIB=$PWD/$L timeout -k 10 200 python -u tools/boot_prof.py > $O/boot_ab.log 2>&1 || { tail -20 $O/boot_ab.log; exit 1; }
    echo "$L $(grep 'call' $O/boot_ab.log | awk '{print $(NF-1)}' | tr '\n' ' ')" | tee -a $out
  done
done
