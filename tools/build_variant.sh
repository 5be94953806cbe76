#!/bin/bash
# Build liblira_hip.so with one csrc file replaced into variants/<name>.so (for
# same-box A/B timing via tools/ab.sh):  tools/build_variant.sh <csrc name> <alt source> <name>
#   e.g. tools/build_variant.sh lira_screen.hip /tmp/screen_qr128.hip qr128
# (VARIANT_FLAGS: extra compile flags, e.g. -DLIRA_PHASE_CLOCKS for tools/phase_clocks.py)
set -e
file=$1; src=$2; name=$3
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/lira-ann-search_amd
make -s -C "$pkg"
mkdir -p "$root/variants/obj_$name"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I$root/include -I$pkg/csrc $VARIANT_FLAGS"
cp "$src" "$pkg/csrc/_variant.hip"
/opt/rocm/bin/hipcc $F -c "$pkg/csrc/_variant.hip" -o "$root/variants/obj_$name/variant.o"
rm -f "$pkg/csrc/_variant.hip"
objs=""
for o in "$pkg"/build/*.o; do
  [ "$(basename "$o" .o).hip" = "$file" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$root/variants/obj_$name/variant.o" -o "$root/variants/$name.so"
echo "built variants/$name.so"
