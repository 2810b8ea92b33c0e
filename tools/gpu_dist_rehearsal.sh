#!/bin/bash
# Rehearse the multi-rank bench on ONE GPU: 2 ranks over RCCL sharing GPU 0 (if RCCL allows
# it), else over gloo; plus the fp exactness GPU test.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/dist; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "fast_sqrt" --timeout 120 --timeout-method thread > $out/pytest_fp.log 2>&1; echo "pytest_fp rc=$?"; tail -1 $out/pytest_fp.log
LRT_BENCH_SAME_GPU=1 NCCL_DEBUG=WARN timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 > $out/rccl2.log 2>&1
rc=$?; echo "rccl 2 ranks on one GPU rc=$rc"; tail -4 $out/rccl2.log | cut -c1-600
if [ $rc -ne 0 ]; then
  LRT_DIST_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 10 --warmup 2 > $out/gloo2.log 2>&1
  echo "gloo 2 ranks rc=$?"; tail -2 $out/gloo2.log | cut -c1-600
fi
