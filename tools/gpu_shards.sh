#!/bin/bash
# Per-GPU render time of rank 0's shard in an N-GPU weak-scaling run, on one GPU.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/shards; mkdir -p $out
for k in ${KERNELS:-v0}; do for n in ${NS:-1 2 4 8}; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --shard-of $n --kernel $k $BENCH_ARGS > $out/s${n}_$k.log 2>&1 || { echo "s$n $k failed"; tail -3 $out/s${n}_$k.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/s${n}_$k.log').read().strip().splitlines()[-1]); print('shard-of $n $k', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms kernel', d['ms_per_step'], 'ms/step')"
done; done
