#!/bin/bash
# BVH paths: GPU parity (BVH == linear scan, 1000-sphere goldens, fuzz), then configs 4 and 3
set -o pipefail
mkdir -p gpurun_out/sah
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_features.py -k "bvh or scene1000 or c4 or c5 or fuzz" > gpurun_out/sah/tests.log 2>&1 || { tail -30 gpurun_out/sah/tests.log; exit 1; }
tail -1 gpurun_out/sah/tests.log
CFGS="sah:6" tools/gpu_sah.sh
