#!/bin/bash
# Build the 8-wide walk simulator (tools/w8sim.cpp, a development tool) against the in-tree
# sources and librtxscene; the binary lands in tools/w8sim (git-ignored).
set -eu
cd "$(dirname "$0")/.."
C=c-raytracer_amd
/opt/rocm/bin/hipcc -std=c++17 -O2 -fopenmp -I include -I $C/csrc -I $C/host tools/w8sim.cpp $C/csrc/rtx_wide8.cpp \
  $C/csrc/bvh_build.cpp $C/csrc/rtx_frame.cpp -o tools/w8sim -L $C/lib -lrtxscene -Wl,-rpath,$PWD/$C/lib
