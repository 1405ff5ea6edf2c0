#!/bin/bash
# Build a variant of libmhmkc.so with extra -D flags into exp/ (performance A/B runs, tools/ab.sh).
#   tools/build_variant.sh NAME [-DMACRO=V ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
  mhm2_proxy_amd/csrc/*.hip mhm2_proxy_amd/csrc/mhmkc_host.cpp \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o exp/libmhmkc_$name.so
echo "built exp/libmhmkc_$name.so $*"
