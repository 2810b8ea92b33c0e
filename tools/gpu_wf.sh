#!/bin/bash
# wavefront (v4) bring-up: parity, then configs 2/3/4 v0 vs wf.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/wf; mkdir -p $out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $out/$name.log; exit $rc; fi; }
show() { python3 -c "import json,sys; d=json.loads(open('$out/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms/launch')"; }
run pytest_wf 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "wavefront or 256" --timeout 120 --timeout-method thread
tail -1 $out/pytest_wf.log
for cfg in ${CONFIGS:-2 3 4}; do
  st=5; [ $cfg = 4 ] && st=2
  run c${cfg}_v0 300 python bench.py --steps $st --warmup 1 --no-cpu-baseline --config $cfg --kernel v0; show c${cfg}_v0
  run c${cfg}_wf 300 python bench.py --steps $st --warmup 1 --no-cpu-baseline --config $cfg --kernel wf; show c${cfg}_wf
done
