#!/bin/bash
# dev tool: libemqx_tm built with extra defines into emqx_amd/variants/
#   tools/build_variant.sh NAME [-DFOO ...]
set -e
name=$1; shift
mkdir -p emqx_amd/variants
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fvisibility=hidden -Wl,-soname,libemqx_tm.so "$@" \
  -o emqx_amd/variants/libemqx_tm_$name.so emqx_amd/csrc/tm_engine.cpp emqx_amd/csrc/tm_group.cpp emqx_amd/csrc/tm_shard.cpp emqx_amd/csrc/tm_kernels.hip -lpthread
