#!/bin/bash
# dev: build a tuning variant of the library, e.g. tools/build_variant.sh seg512 -DRDF_LIGHT_SEG=512
# -> rdfind_amd/librdfind_hip_<name>.so (loaded with RDFIND_HIP_LIB=...)
set -e
cd "$(dirname "$0")/../rdfind_amd/csrc"
NAME=$1; shift
mkdir -p build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c rdfind_hip.hip -o build/rdfind_hip_$NAME.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../librdfind_hip_$NAME.so build/primitives.o build/rdfind_hip_$NAME.o
