#!/bin/bash
# v3 (path regeneration) bring-up: parity tests of v3, then config 2/3/4 timings of v0 vs v3
# at several regeneration thresholds.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/v3; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "$out/$name.log"; exit $rc; fi
}
step pytest_v3 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "v3 or variants or bvh_equals" --timeout 120 --timeout-method thread
tail -2 $out/pytest_v3.log
show() { python3 -c "import json,sys; d=json.loads(open('$out/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms/launch')"; }
for cfg in ${CONFIGS:-2 3}; do
  step c${cfg}_v0 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel v0; show c${cfg}_v0
  for m in ${MINS:-8 16 24 32}; do
    LRT_V3_REGEN_MIN=$m step c${cfg}_v3_m$m 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel v3; show c${cfg}_v3_m$m
  done
done
