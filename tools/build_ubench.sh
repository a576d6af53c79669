#!/bin/bash
# Build the diagnostic micro-benchmarks (tools/bin/), gfx950.
set -e
cd "$(dirname "$0")"
mkdir -p bin
for f in ubench_chol ubench_fp64 ubench_lat repro_coop_exit; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bin/$f $f.hip
done
