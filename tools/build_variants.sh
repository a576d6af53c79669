#!/bin/bash
# Build A/B variants of libm3s_backend.so with different compile-time knobs into
# mast3r-slam_amd/lib/variants/<name>.so (select one with M3S_BACKEND_LIB=...).
# usage: [ONLY="gn_accum ..."] tools/build_variants.sh name1 "-DFOO=1" name2 "-DFOO=2" ...
# ONLY: recompile just these sources with the variant's flags and link them with the normal
# build's objects of the others (run `make` first).  SRC_<file>=path swaps in another source.
set -e
cd "$(dirname "$0")/../mast3r-slam_amd"
mkdir -p lib/variants build/variants
all=$(sed -n 's/^SRCS := //p' Makefile | sed 's|csrc/||g; s|\.hip||g')
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    objs=""
    pids=""
    for f in $all; do
        if [ -n "${ONLY:-}" ] && ! echo " $ONLY " | grep -q " $f "; then
            objs="$objs build/$f.o"
            continue
        fi
        fc=-ffp-contract=fast-honor-pragmas
        case $f in matching|match_glue|edges|keyframe|gn_refacc) fc=-ffp-contract=off ;; esac
        [ $f = gn_accum ] && fc="$fc -fno-slp-vectorize"
        src=csrc/$f.hip
        ov=SRC_$f
        [ -n "${!ov:-}" ] && src=${!ov}
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Icsrc -I../include $fc $flags \
            -c $src -o build/variants/${name}_$f.o &
        pids="$pids $!"
        objs="$objs build/variants/${name}_$f.o"
    done
    for p in $pids; do wait $p; done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/variants/$name.so $objs -ldl
    echo "built lib/variants/$name.so ($flags)"
done
