#!/bin/bash
# Build liblira_hip.so with an alternative lira_scan.hip into variants/<name>.so
# (for same-box A/B timing via LIRA_HIP_LIB=variants/<name>.so).
set -e
src=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/lira-ann-search_amd
mkdir -p "$root/variants/obj_$name"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I$root/include -I$pkg/csrc"
cp "$src" "$pkg/csrc/_variant_scan.hip"
/opt/rocm/bin/hipcc $F -c "$pkg/csrc/_variant_scan.hip" -o "$root/variants/obj_$name/scan.o"
rm -f "$pkg/csrc/_variant_scan.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$pkg/build/lira_abi.o" "$root/variants/obj_$name/scan.o" \
    "$pkg/build/lira_rank.o" "$pkg/build/lira_build.o" -o "$root/variants/$name.so"
echo "built variants/$name.so"
