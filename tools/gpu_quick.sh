#!/bin/bash
# Quick iteration loop: GPU parity suite, bench (v1 + optional extra args), SQ counters of v1.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/q/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; tail -20 "gpurun_out/q/$name.log"; exit $rc; fi
  return 0
}
step pytest_gpu 420 python -m pytest tests -m gpu -q -p no:cacheprovider -x
tail -3 gpurun_out/q/pytest_gpu.log
for cfg in ${CONFIGS:-2}; do
  step bench_c$cfg 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg $BENCH_ARGS
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/q/bench_c$cfg.log').read().strip().splitlines()[-1]); print('config$cfg', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms/launch', d['config'].get('kernel'))"
done
export TMPDIR=/tmp
CNT="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY"
step pmc 300 rocprofv3 --pmc $CNT -d gpurun_out/q -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS
python3 - <<'PY'
import csv, collections
agg=collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/q/pmc_counter_collection.csv')):
    if 'paths' in r['Kernel_Name'] or 'trace_kernel' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
a={c: sum(v)/len(v) for c,v in agg.items()}
print({c: '%.4g'%v for c,v in a.items()})
if 'SQ_THREAD_CYCLES_VALU' in a: print('VALU lane utilisation %.1f%%' % (100*a['SQ_THREAD_CYCLES_VALU']/(a['SQ_ACTIVE_INST_VALU']*64)))
PY
