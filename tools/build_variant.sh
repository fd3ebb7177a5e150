#!/bin/bash
# A/B variant of the native library (diagnostic, never the shipped build):
#   tools/build_variant.sh <name> <file.hip> [-DFOO=1 ...]
# recompiles <file.hip> with the extra defines, links it with the other
# objects of the regular build (csrc/build/), and writes
# deeprank2_amd/libdeeprank2_amd_<name>.so, selected at run time by DR_LIB_NAME.
set -e
cd "$(dirname "$0")/../deeprank-gnn-2_amd/csrc"
name=$1; src=$2; shift 2
make -s >/dev/null
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -c "$src" -o "build_var/$name.$src.o"
objs=$(ls build/*.o | grep -v "build/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../deeprank2_amd/libdeeprank2_amd_$name.so" $objs "build_var/$name.$src.o"
echo "built libdeeprank2_amd_$name.so"
