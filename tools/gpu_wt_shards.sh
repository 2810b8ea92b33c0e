cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wt
for n in 1 8; do
  rm -f gpurun_out/wt/s$n.bin
  LRT_LIB=$PWD/build_exp/liblrt_WT.so LRT_WAVETRACE=gpurun_out/wt/s$n.bin timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard-of $n > gpurun_out/wt/s$n.log 2>&1 || { echo fail; tail -3 gpurun_out/wt/s$n.log; exit 1; }
  echo "== shard-of $n"; python3 tools/wavetrace.py gpurun_out/wt/s$n.bin
done
