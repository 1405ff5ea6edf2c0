#!/bin/bash
# Build a variant of libmhmkc.so with extra -D flags into exp/ (performance A/B runs, tools/ab.sh).
#   tools/build_variant.sh NAME [-DMACRO=V ...]
set -e
cd "$(dirname "$0")/.."
python -m mhm2_proxy_amd.build --variant "$@"
