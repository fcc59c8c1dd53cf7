#!/bin/bash
# Build a library variant of the current tree for same-box A/B runs
# (tools/gpu_ab_libs.sh): tools/build_ab_lib.sh NAME -DMACRO=V ...
#   -> ab/lib/libyrss_NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p ab/lib
C=yastack_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result \
    -Wno-pass-failed -DYRSS_TOOLS_BUILD=1 "$@" -I include $C/yrss.hip $C/yrss_pcap.cpp $C/yrss_shard.cpp $C/yrss_fanout.cpp \
    -o ab/lib/libyrss_$name.so
echo "built ab/lib/libyrss_$name.so"
