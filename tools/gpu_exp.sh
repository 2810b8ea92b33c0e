#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-STAMPS NOIO STATIC BOTH}; do
  export LRT_LIB=$PWD/build_exp/liblrt_$v.so
  echo "== $v"
  timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu-baseline 2> gpurun_out/exp_$v.err | cut -c1-120 || { echo "$v failed"; exit 1; }
  grep stamps gpurun_out/exp_$v.err
done
