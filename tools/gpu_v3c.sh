#!/bin/bash
# v3 round 2: parity of the lean v3, timings, per-section stats (SEC build), fp exactness probe.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/v3c; mkdir -p $out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $out/$name.log; exit $rc; fi; }
show() { python3 -c "import json,sys; d=json.loads(open('$out/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms/launch')"; }
run pytest_v3 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "v3 or variants or bvh_equals" --timeout 120 --timeout-method thread
tail -1 $out/pytest_v3.log
for cfg in 2 3; do
  run c${cfg}_v0 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel v0; show c${cfg}_v0
  for m in 8 16 32; do
    LRT_V3_REGEN_MIN=$m run c${cfg}_v3_m$m 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel v3; show c${cfg}_v3_m$m
  done
done
LRT_LIB=build_exp/liblrt_SEC.so run sec_v0 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --kernel v0
grep secstats $out/sec_v0.log | tail -9
LRT_LIB=build_exp/liblrt_SEC.so LRT_V3_REGEN_MIN=16 run sec_v3 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --kernel v3
grep secstats $out/sec_v3.log | tail -9
run fpexact 300 tools/fpexact
cat $out/fpexact.log
