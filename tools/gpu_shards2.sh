#!/bin/bash
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/shards2; mkdir -p $out
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms kernel', d['config']['rays_per_step'], 'rays')"; }
b full_spp4 --spp 4
b full_spp8 --spp 8
b full_spp16 --spp 16
b full_spp32 --spp 32
b shard8_rb8 --shard-of 8
b shard8_rb1 --shard-of 8 --row-block 1
b shard8_rb90 --shard-of 8 --row-block 90
b shard2_spp4 --shard-of 2 --spp 2
b shard8_spp4 --shard-of 8 --spp 1
