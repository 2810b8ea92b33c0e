#!/bin/bash
# Full evidence run for the default bench config: bench (with CPU baseline), rocprofv3 kernel
# trace + stats, and PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) in separate runs.
# Usage: TAG=r1_v3 [BENCH_ARGS=...] bash tools/gpu_profile_round.sh
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-latest}
out=gpurun_out/$TAG; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi; }
run bench 300 python bench.py --steps 20 --warmup 3 $BENCH_ARGS
tail -1 $out/bench.log > $out/bench.json
run trace 300 rocprofv3 --kernel-trace --stats -d $out -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS
run trace1 300 rocprofv3 --kernel-trace --stats -d $out -o trace1 --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 $BENCH_ARGS
run fetch 300 rocprofv3 --pmc FETCH_SIZE -d $out -o pmc_fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $BENCH_ARGS
run write 300 rocprofv3 --pmc WRITE_SIZE -d $out -o pmc_write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $BENCH_ARGS
run sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY -d $out -o pmc_sq --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $BENCH_ARGS
cat $out/bench.json | cut -c1-300
