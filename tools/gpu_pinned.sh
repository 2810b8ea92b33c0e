#!/bin/bash
# host-buffer paths: DrawTest/render_host parity (pageable, pinned, lrt_host_alloc), then rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "draw_test or pinned or host_alloc or alpha" > gpurun_out/pinned_tests.log 2>&1 || { tail -30 gpurun_out/pinned_tests.log; exit 1; }
tail -1 gpurun_out/pinned_tests.log
timeout -k 10 120 python -u tools/drawtest_rate.py 200 | tee gpurun_out/pinned_rate.log
timeout -k 10 120 python -u tools/drawtest_rate.py 200 pinned | tee -a gpurun_out/pinned_rate.log
