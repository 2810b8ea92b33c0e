#!/bin/bash
# v3 diagnosis: SQ counters of v0 and v3 (config 2) and v3 timings at high thresholds.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/v3b; mkdir -p $out
export TMPDIR=/tmp
G4="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
G1="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM"
run() { local name=$1; shift; timeout -k 10 200 "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi; }
for k in v0 v3; do
  for m in 16 64; do
    [ $k = v0 ] && [ $m = 64 ] && continue
    export LRT_V3_REGEN_MIN=$m
    run ${k}m${m}_g4 rocprofv3 --pmc $G4 -d $out -o ${k}m${m}_g4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --kernel $k
    run ${k}m${m}_g1 rocprofv3 --pmc $G1 -d $out -o ${k}m${m}_g1 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --kernel $k
  done
done
python3 tools/counter_table.py $out
show() { python3 -c "import json,sys; d=json.loads(open('$out/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms/launch')"; }
for m in 40 48 56 64; do
  LRT_V3_REGEN_MIN=$m run t_m$m python bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel v3; show t_m$m
done
