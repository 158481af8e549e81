#!/bin/bash
# Build an alternate libtapeec (varlib/lib_<name>.so) with one kernel source (default
# encode_dma.hip) compiled with extra -D flags, for A/B timing through TAPE_EC_LIB
# (scripts/gpu_enc_ab2.sh).  Needs tape_amd/build/*.o.
#   bash scripts/build_var.sh slp3 "-DTEC_DMA_WPE=3" [decode_stage.hip]
set -e
cd "$(dirname "$0")/.."
name=$1; defs=$2; src=${3:-encode_dma.hip}
mkdir -p varlib/build_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wall -Wno-unused-result $defs -c -o varlib/build_$name/$src.o tape_amd/csrc/$src
objs=$(ls tape_amd/build/*.o tape_amd/build/gen/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o varlib/lib_$name.so $objs varlib/build_$name/$src.o -L/opt/rocm/lib -lhiprtc
echo built varlib/lib_$name.so
