#!/bin/bash
# Build A/B variants of libm3s_backend.so with different compile-time knobs into
# mast3r-slam_amd/lib/variants/<name>.so (select one with M3S_BACKEND_LIB=...).
# usage: tools/build_variants.sh name1 "-DFOO=1" name2 "-DFOO=2" ...
set -e
cd "$(dirname "$0")/../mast3r-slam_amd"
mkdir -p lib/variants build/variants
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    objs=""
    for f in $(sed -n 's/^SRCS := //p' Makefile | sed 's|csrc/||g; s|\.hip||g'); do
        fc=-ffp-contract=fast-honor-pragmas
        case $f in matching|match_glue|edges|keyframe|gn_refacc) fc=-ffp-contract=off ;; esac
        [ $f = gn_accum ] && fc="$fc -fno-slp-vectorize"
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Icsrc -I../include $fc $flags \
            -c csrc/$f.hip -o build/variants/${name}_$f.o
        objs="$objs build/variants/${name}_$f.o"
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/variants/$name.so $objs -ldl
    echo "built lib/variants/$name.so ($flags)"
done
