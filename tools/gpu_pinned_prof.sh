#!/bin/bash
# kernel + memory-copy trace of the DrawTest host path with a page-locked buffer (zero copy)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p $R/gpurun_out/pprof
LRT_HOST_CHUNKS=0 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/pprof/zc -o run -- python3 $R/tools/drawtest_rate.py 50 pinned > $R/gpurun_out/pprof/zc.log 2>&1 || exit 1
