#!/bin/bash
# sample mode: parity (auto and forced) and shard timings with it off / auto.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/samp; mkdir -p $out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $out/$name.log; exit $rc; fi; }
run pytest_auto 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
tail -1 $out/pytest_auto.log
LRT_SAMPLE_MODE=2 run pytest_forced 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
tail -1 $out/pytest_forced.log
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms kernel', d['ms_per_step'], 'ms/step')"; }
for m in 0 1; do for n in 1 2 4 8; do LRT_SAMPLE_MODE=$m b m${m}_s$n --shard-of $n; done; done
LRT_SAMPLE_MODE=1 b m1_c3 --config 3
