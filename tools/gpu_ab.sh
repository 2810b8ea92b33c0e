#!/bin/bash
# bench several kernels back to back: KERNELS="v0 v2 v2s" CONFIGS="2 3"
cd "$GRAFT_REPO_ROOT"
for cfg in ${CONFIGS:-2}; do for k in ${KERNELS:-v0 v2}; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel $k > gpurun_out/ab_${cfg}_$k.log 2>&1 || { echo "$cfg $k failed"; tail -3 gpurun_out/ab_${cfg}_$k.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_${cfg}_$k.log').read().strip().splitlines()[-1]); print('config$cfg', '$k', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms')"
done; done
