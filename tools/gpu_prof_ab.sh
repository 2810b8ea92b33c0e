#!/bin/bash
# A/B counters for v0 vs v1 kernels.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/ab/counters_list.txt 2>&1 || true
CNT="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY"
for k in v0 v1; do
  timeout -k 10 300 rocprofv3 --pmc $CNT -d gpurun_out/ab -o pmc_$k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel $k > gpurun_out/ab/bench_$k.log 2>&1
  rc=$?; echo "$k rc=$rc"; if [ $rc -ne 0 ]; then tail gpurun_out/ab/bench_$k.log; exit $rc; fi
done
