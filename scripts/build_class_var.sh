#!/bin/bash
# Build an alternate libtapeec (varlib/lib_<name>.so) whose decode class kernels are generated with
# build-time options (dec_class.hpp DecClassGenOpt), for A/B timing through TAPE_EC_LIB.
#   bash scripts/build_class_var.sh late "TEC_GEN_LATE=1"     (needs tape_amd/build/*.o)
set -e
cd "$(dirname "$0")/.."
name=$1; envs=$2
d=/tmp/varlib_gen_$name
mkdir -p $d
env $envs tape_amd/build/gen_dec_class $d
ls $d/dec_class_[0-9]*.hip | xargs -P 8 -I{} /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Wno-unused-variable -Itape_amd/csrc -c -o {}.o {}
objs=$(ls tape_amd/build/*.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o varlib/lib_$name.so $objs $d/*.hip.o -L/opt/rocm/lib -lhiprtc
echo built varlib/lib_$name.so
