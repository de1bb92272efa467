#!/bin/bash
# Builds kernel performance variants into truetrace-unity-pathtracer_amd/lib/variants/.
# Each line: NAME FLAGS...
cd "$(dirname "$0")/.." || exit 1
PKG=truetrace-unity-pathtracer_amd
build() { name=$1; shift; make -s -C $PKG variant NAME=$name VFLAGS="$*" > /tmp/variant_$name.log 2>&1 || { echo "FAILED $name"; cat /tmp/variant_$name.log; }; }
while read -r name flags; do
  [ -z "$name" ] && continue
  build $name $flags &
done < "${1:-tools/variants.txt}"
wait
ls $PKG/lib/variants
