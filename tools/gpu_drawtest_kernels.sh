cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dt
for k in v0 v3 wf; do for d in 8 20; do
  for m in 8 16; do
    [ $k != v3 ] && [ $m = 16 ] && continue
    LRT_V3_REGEN_MIN=$m timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spp 1 --depth $d --kernel $k > gpurun_out/dt/${k}_d${d}_m$m.log 2>&1 || { echo fail $k; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/dt/${k}_d${d}_m$m.log').read().strip().splitlines()[-1]); print('$k depth $d m$m', d['value'], 'Mray/s', d['roofline']['kernel_ms'], 'ms')"
  done
done; done
