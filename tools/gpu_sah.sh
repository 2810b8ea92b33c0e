#!/bin/bash
# BVH build A/B on config 4: split (sah / median) x leaf size
set -o pipefail
mkdir -p gpurun_out/sah
for cfg in ${CFGS:-sah:5 sah:6 sah:8 sah:10 sah:12 sah:16}; do
  m=${cfg%:*}; l=${cfg#*:}
  LRT_BVH_SPLIT=$m LRT_BVH_LEAF=$l timeout -k 10 200 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sah/c4_${m}_$l.log 2>&1 || { tail -5 gpurun_out/sah/c4_${m}_$l.log; exit 1; }
  grep '^{' gpurun_out/sah/c4_${m}_$l.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'])"
done
