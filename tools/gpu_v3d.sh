#!/bin/bash
# v3 group regeneration: parity + timings (+ SQ counters of v3 on config 2).
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/v3d; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $out/$name.log; exit $rc; fi; }
show() { python3 -c "import json,sys; d=json.loads(open('$out/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms/launch')"; }
run pytest_v3 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "v3 or variants or bvh_equals" --timeout 120 --timeout-method thread
tail -1 $out/pytest_v3.log
for cfg in ${CONFIGS:-2 3}; do
  run c${cfg}_v0 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel v0; show c${cfg}_v0
  for m in ${MINS:-4 8 16 32}; do
    LRT_V3_REGEN_MIN=$m run c${cfg}_v3_m$m 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel v3; show c${cfg}_v3_m$m
  done
done
if [ -n "$SEC" ]; then
LRT_LIB=build_exp/liblrt_SEC.so LRT_V3_REGEN_MIN=${SECMIN:-8} run sec_v3 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --kernel v3
grep secstats $out/sec_v3.log | tail -9
fi
G4="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
LRT_V3_REGEN_MIN=${SECMIN:-8} run v3_g4 200 rocprofv3 --pmc $G4 -d $out -o v3_g4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --kernel v3
python3 tools/counter_table.py $out
