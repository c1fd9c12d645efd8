#!/bin/bash
# Measurement builds: libgeohip_<name>.so = the product objects with one source recompiled under
# extra defines (an ablation or an alternative kept out of the product).
#   scripts/build_variant.sh <name> <source.hip> -DFLAG ...
#   VARIANT_SRC=/tmp/old.hip scripts/build_variant.sh old cell_kernels.hip   (another text of that source)
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
python3 -c "import sys; sys.path.insert(0, '.'); from spatialflink_amd import build; build.build()" >/dev/null
mkdir -p build/variant
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -Iinclude \
    -Ispatialflink_amd/csrc -x hip --offload-arch=gfx950 "$@" -c ${VARIANT_SRC:-spatialflink_amd/csrc/$src} -o build/variant/$name.o
objs=$(ls build/geohip/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/variant/$name.o -o spatialflink_amd/libgeohip_$name.so
echo spatialflink_amd/libgeohip_$name.so
