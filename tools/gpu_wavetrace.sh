#!/bin/bash
# wave-lifetime traces: VARIANTS="WT WT_S1" CONFIGS="2 3" bash tools/gpu_wavetrace.sh
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-WT}; do for cfg in ${CONFIGS:-2}; do
  rm -f gpurun_out/wt_${v}_$cfg.bin
  LRT_LIB=$PWD/build_exp/liblrt_$v.so LRT_WAVETRACE=gpurun_out/wt_${v}_$cfg.bin timeout -k 10 200 \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --config $cfg --kernel ${KERNEL:-v0} > gpurun_out/wt_${v}_$cfg.log 2>&1 \
    || { echo "$v $cfg failed"; tail -3 gpurun_out/wt_${v}_$cfg.log; exit 1; }
  echo "== $v config$cfg"; python3 tools/wavetrace.py gpurun_out/wt_${v}_$cfg.bin
done; done
