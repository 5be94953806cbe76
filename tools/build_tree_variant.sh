#!/bin/bash
# Build the working tree's csrc/ (optionally with one file replaced) into
# variants/<name>.so, leaving the in-tree library alone (same-box A/B via tools/ab.sh).
#   tools/build_tree_variant.sh <name> [<csrc file> <alt source>]   (VARIANT_FLAGS: extra flags)
set -e
name=$1; file=$2; src=$3
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/lira-ann-search_amd
out=$root/variants/obj_$name
mkdir -p "$out"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I$root/include -I$pkg/csrc $VARIANT_FLAGS"
objs=""
for s in "$pkg"/csrc/*.hip; do
  b=$(basename "$s")
  [ "$b" = _variant.hip ] && continue
  if [ -n "$file" ] && [ "$b" = "$file" ]; then
    cp "$src" "$pkg/csrc/_variant.hip"; s="$pkg/csrc/_variant.hip"
  fi
  /opt/rocm/bin/hipcc $F -c "$s" -o "$out/${b%.hip}.o" &
  objs="$objs $out/${b%.hip}.o"
done
wait
rm -f "$pkg/csrc/_variant.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o "$root/variants/$name.so"
echo "built variants/$name.so"
