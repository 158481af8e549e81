#!/bin/bash
# Build an alternate libtapeec (varlib/lib_<name>.so) whose encode_dma.hip is compiled with extra
# -D flags, for A/B timing through TAPE_EC_LIB (scripts/gpu_libvar.sh).  Needs tape_amd/build/*.o.
#   bash scripts/build_var.sh slp3 "-DTEC_DMA_WPE=3"
set -e
cd "$(dirname "$0")/.."
name=$1; defs=$2
mkdir -p varlib/build_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-result $defs -c -o varlib/build_$name/encode_dma.hip.o tape_amd/csrc/encode_dma.hip
objs=$(ls tape_amd/build/*.o | grep -v encode_dma)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o varlib/lib_$name.so $objs varlib/build_$name/encode_dma.hip.o -L/opt/rocm/lib -lhiprtc
echo built varlib/lib_$name.so
