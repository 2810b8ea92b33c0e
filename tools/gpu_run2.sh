#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace + PMC passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: stop the session on crash/timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_gpu 420 python -m pytest tests -m gpu -q -p no:cacheprovider
tail -4 gpurun_out/pytest_gpu.log
step bench 300 python bench.py --steps 20 --warmup 3
tail -1 gpurun_out/bench.log
step bench_global 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --scene-global
tail -1 gpurun_out/bench_global.log
export TMPDIR=/tmp
step prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof -o pmc_fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
step prof_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof -o pmc_write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
step prof_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/prof -o pmc_sq --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
find gpurun_out/prof -name "*.csv" | head -20
