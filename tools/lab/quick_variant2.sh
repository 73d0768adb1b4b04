#!/bin/bash
# Variant library that differs from the main build only in the listed
# translation units: reuse build/obj, rebuild those objects with extra flags.
# usage: tools/lab/quick_variant2.sh <name> "<units>" <-D flags...>
set -eu
NAME=$1; UNITS=$2; shift 2
cd "$(dirname "$0")/../../node-fhe-accelerate_amd"
rm -rf build/obj_$NAME && mkdir -p build/obj_$NAME && cp -p build/obj/*.o build/obj_$NAME/
for u in $UNITS; do rm -f build/obj_$NAME/$u.o; done
make -s -j8 VARIANT=_$NAME EXTRA="$*" > /dev/null
echo "built build/libfhe_gpu_$NAME.so ($UNITS: $*)"
