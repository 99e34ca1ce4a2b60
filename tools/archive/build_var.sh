#!/bin/bash
# A/B library variants: build_var.sh <name> <file.hip> <extra hipcc flags...>
# recompiles one kernel file with extra flags and links it with the other objects of the
# current build into ransac_amd/build_var/lib_<name>.so
set -e
cd "$(dirname "$0")/../../ransac_amd"
NAME=$1; SRC=$2; shift 2
mkdir -p build_var var_libs
OBJ=build/$(basename $SRC .hip).o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result \
    -I/opt/rocm/include "$@" -c csrc/$SRC -o build_var/$NAME.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 build_var/$NAME.o $(ls build/*.o | grep -v "^$OBJ$") \
    -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o var_libs/lib_$NAME.so
rm build_var/$NAME.o
