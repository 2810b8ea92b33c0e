#!/bin/bash
# bench steps over 1 / 2 / 3 render streams, N=1 and rank 0's 8-GPU shard; 2-rank gloo run.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/streams; mkdir -p $out
show() { python3 -c "import json,sys; d=json.loads(open('$out/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms kernel', d['ms_per_step'], 'ms/step')"; }
for st in 1 2 3; do
  for sh in 1 8; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams $st --shard-of $sh > $out/s${st}_sh$sh.log 2>&1 || { echo fail; tail -3 $out/s${st}_sh$sh.log; exit 1; }
    show s${st}_sh$sh
  done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 2 --config 3 > $out/c3.log 2>&1 && show c3
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/dist.log 2>&1; echo "dist rc=$?"; tail -1 $out/dist.log
