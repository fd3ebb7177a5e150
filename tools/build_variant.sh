#!/bin/bash
# A/B variant of the native library (diagnostic, never the shipped build):
#   tools/build_variant.sh <name> <file.hip>[,<file.hip>...] [-DFOO=1 ...]
# recompiles the listed sources with the extra defines, links them with the
# other objects of the regular build (csrc/build/), and writes
# deeprank2_amd/libdeeprank2_amd_<name>.so, selected at run time by DR_LIB_NAME.
set -e
cd "$(dirname "$0")/../deeprank-gnn-2_amd/csrc"
name=$1; srcs=$2; shift 2
make -s >/dev/null
mkdir -p build_var
objs=$(ls build/*.o)
var=""
for src in ${srcs//,/ }; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -c "$src" -o "build_var/$name.$src.o"
  objs=$(echo "$objs" | grep -v "build/$src.o")
  var="$var build_var/$name.$src.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../deeprank2_amd/libdeeprank2_amd_$name.so" $objs $var
echo "built libdeeprank2_amd_$name.so"
