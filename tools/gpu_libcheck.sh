#!/bin/bash
# A/B of library builds with a parity subset per build: LIBS="default NOFS FR" CONFIGS="2 3"
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/libcheck; mkdir -p $out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $out/$name.log; exit $rc; fi; }
if [ -x tools/fpexact ]; then run fpexact 300 tools/fpexact; grep -v "    e=" $out/fpexact.log; fi
for lib in ${LIBS:-default}; do
  if [ $lib = default ]; then unset LRT_LIB; else export LRT_LIB=$PWD/build_exp/liblrt_$lib.so; fi
  run parity_$lib 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "${PARITY_K:-config2_full or golden_fuzz or golden_mode_p or scene1000 or config3_rows}" --timeout 120 --timeout-method thread
  tail -1 $out/parity_$lib.log
  for cfg in ${CONFIGS:-2}; do
    run b_${lib}_$cfg 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --config $cfg ${BENCH_ARGS}
    python3 -c "import json; d=json.loads(open('$out/b_${lib}_$cfg.log').read().strip().splitlines()[-1]); print('$lib', 'config$cfg', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms')"
  done
done
