#!/bin/bash
# Build the product library as of git revision REV into build_exp/liblrt_<NAME>.so (A/B
# against the working tree): bash tools/build_rev.sh PREV HEAD [-DFLAGS...]
# (revisions before the round-4 split into translation units had one lrt_hip.hip)
set -e
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" learnraytracing_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/build_exp"
cd "$tmp/learnraytracing_amd/csrc"
if [ -f lrt_hip.hip ]; then
  /opt/rocm/bin/hipcc -O3 "$@" -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -I../../include \
    -Wall -Wno-unused-function -shared -o "$root/build_exp/liblrt_$name.so" lrt_hip.hip $(ls lrt_sort.hip 2>/dev/null) \
    -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
else
  make -j16 EXTRA="$*" LIB="$root/build_exp/liblrt_$name.so" "$root/build_exp/liblrt_$name.so"
fi
rm -rf "$tmp"
echo "built build_exp/liblrt_$name.so ($rev $*)"
