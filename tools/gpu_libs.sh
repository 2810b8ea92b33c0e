#!/bin/bash
# bench kernels x library builds: LIBS="default W5 W6" KERNELS="v0 v2s" CONFIGS="2"
cd "$GRAFT_REPO_ROOT"
for lib in ${LIBS:-default}; do
  if [ $lib = default ]; then unset LRT_LIB; else export LRT_LIB=$PWD/build_exp/liblrt_$lib.so; fi
  for cfg in ${CONFIGS:-2}; do for k in ${KERNELS:-v0 v2s}; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config $cfg --kernel $k > gpurun_out/lib_${lib}_${cfg}_$k.log 2>&1 || { echo "$lib $cfg $k failed"; tail -3 gpurun_out/lib_${lib}_${cfg}_$k.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/lib_${lib}_${cfg}_$k.log').read().strip().splitlines()[-1]); print('$lib', 'config$cfg', '$k', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms')"
  done; done
done
