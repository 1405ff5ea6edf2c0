#!/bin/bash
# Build libmhmkc.so from a committed revision (default HEAD) into exp/libmhmkc_0prev.so, the reference
# arm of a tools/ab.sh performance A/B against the working tree.
#   tools/build_prev.sh [REV]
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
tmp=$(mktemp -d)
mkdir -p "$tmp/mhm2_proxy_amd/csrc" "$tmp/include" exp
for f in $(git ls-tree -r --name-only "$rev" mhm2_proxy_amd/csrc include); do
  mkdir -p "$tmp/$(dirname "$f")"
  git show "$rev:$f" > "$tmp/$f"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$tmp"/mhm2_proxy_amd/csrc/*.hip \
  "$tmp"/mhm2_proxy_amd/csrc/mhmkc_host.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o exp/libmhmkc_0prev.so
rm -rf "$tmp"
echo "built exp/libmhmkc_0prev.so from $rev"
