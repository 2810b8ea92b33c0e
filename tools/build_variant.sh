#!/bin/bash
# Build an A/B variant of the product library into build_exp/liblrt_<NAME>.so:
#   bash tools/build_variant.sh S1 -DLRT_MAX_SPLIT=1
# then on the GPU: LIBS="default S1" KERNELS=v0 CONFIGS=2 bash tools/gpu_libs.sh
set -e
name=$1; shift
cd "$(dirname "$0")/../learnraytracing_amd/csrc"
mkdir -p ../../build_exp
/opt/rocm/bin/hipcc -O3 "$@" -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../../include \
  -Wall -Wno-unused-function -DLRT_ROCTX=1 -shared -o ../../build_exp/liblrt_$name.so lrt_hip.hip $(ls lrt_sort.hip 2>/dev/null) -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "built build_exp/liblrt_$name.so ($*)"
