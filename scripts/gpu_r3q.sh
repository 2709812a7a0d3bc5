#!/bin/bash
# Allocator-poisoning probe of the data-parallel AutoEncoder step (scripts/debug/dp_repeat.py)
mkdir -p gpurun_out
: > gpurun_out/r3q.txt
for np_ in 2 1; do
  for pv in 0 3000 nan; do
    echo "nproc $np_ poison $pv" >> gpurun_out/r3q.txt
    DP_NPROC=$np_ AST_POISON=$pv timeout -k 10 200 python -u scripts/debug/dp_repeat.py 1 gpurun_out >> gpurun_out/r3q.txt 2>&1 || exit 1
  done
done
rm -f gpurun_out/dp_*.npz
