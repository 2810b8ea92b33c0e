#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt; rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err
exit $rc
