#!/bin/bash
# host-buffer paths: DrawTest/render_host parity per LRT_HOST_ZEROCOPY mode (1 = zero copy, 0 = staged), then rates
set -o pipefail
mkdir -p gpurun_out
for z in 1 0; do
  LRT_HOST_ZEROCOPY=$z timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "draw_test or pinned or host_alloc or alpha or non_finite or many_frames" > gpurun_out/pinned_tests$z.log 2>&1 || { tail -30 gpurun_out/pinned_tests$z.log; exit 1; }
  echo "mode $z: $(tail -1 gpurun_out/pinned_tests$z.log)"
done
timeout -k 10 120 python -u tools/drawtest_rate.py 200 | tee gpurun_out/pinned_rate.log
for z in 1 0; do
  LRT_HOST_ZEROCOPY=$z timeout -k 10 120 python -u tools/drawtest_rate.py 200 pinned | sed "s/^/mode=$z /" | tee -a gpurun_out/pinned_rate.log || exit 1
done
