#!/bin/bash
# frame split policy A/B: per-GPU shard times at N=1..8 and configs 3/4, per library build.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/split; mkdir -p $out
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms kernel')"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; echo "pytest rc=$?"; tail -1 $out/pytest.log
for lib in ${LIBS:-MS4 default MS16}; do
  if [ $lib = default ]; then unset LRT_LIB; else export LRT_LIB=$PWD/build_exp/liblrt_$lib.so; fi
  for n in 1 2 4 8; do b ${lib}_s$n --shard-of $n; done
  b ${lib}_c3 --config 3
  STEPS=2 b ${lib}_c4 --config 4
done
