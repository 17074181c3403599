#!/bin/bash
# Build tools/hbm_calib (the HBM counter calibration program) for gfx950, in-tree, on the CPU side.
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 hbm_calib.hip -o bin/hbm_calib
