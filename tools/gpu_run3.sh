#!/bin/bash
# Parity + A/B bench of v0 (LRT_F_SIMPLE) vs v1, plus kernel trace of v1.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_gpu 420 python -m pytest tests -m gpu -q -p no:cacheprovider
tail -4 gpurun_out/pytest_gpu.log
step bench_v1 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
tail -1 gpurun_out/bench_v1.log | cut -c1-400
step bench_v1_c3 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --config 3
tail -1 gpurun_out/bench_v1_c3.log | cut -c1-400
step bench_v1_c4 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --config 4
tail -1 gpurun_out/bench_v1_c4.log | cut -c1-400
export TMPDIR=/tmp
step prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
cat gpurun_out/prof3/trace_kernel_stats.csv | cut -c1-200
