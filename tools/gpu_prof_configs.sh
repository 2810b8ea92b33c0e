#!/bin/bash
# rocprofv3 kernel traces of configs 3 and 4 (bench), for profiles/<TAG>/config{3,4}_*.csv
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-latest}; out=gpurun_out/$TAG; mkdir -p $out
export TMPDIR=/tmp
for cfg in 3 4; do
  st=10; [ $cfg = 4 ] && st=2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o c$cfg --output-format csv -- python3 bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > $out/c$cfg.log 2>&1
  rc=$?; echo "config $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/c$cfg.log; exit $rc; }
  grep "^{" $out/c$cfg.log > $out/c${cfg}_bench.json
  head -3 $out/c${cfg}_kernel_stats.csv | cut -c1-160
done
