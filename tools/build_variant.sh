#!/bin/bash
# Build an A/B variant of the product library into build_exp/liblrt_<NAME>.so:
#   bash tools/build_variant.sh S1 -DLRT_EXP_SECSTATS
# (its objects go to learnraytracing_amd/csrc/_obj_<NAME>), then on the GPU:
#   TAG=x bash tools/gpu.sh ab=S1,4     (tools/gpu.sh: LRT_LIB=build_exp/liblrt_S1.so)
set -e
name=$1; shift
cd "$(dirname "$0")/../learnraytracing_amd/csrc"
mkdir -p ../../build_exp
make -j16 VARIANT="_$name" EXTRA="$*" LIB="../../build_exp/liblrt_$name.so" "../../build_exp/liblrt_$name.so"
echo "built build_exp/liblrt_$name.so ($*)"
