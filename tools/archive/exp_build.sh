#!/bin/bash
# Build experiment variants of librtamd.so (dev tool, run here on the CPU):
#   bash tools/archive/exp_build.sh NAME "-DFLAG ..." [NAME "-DFLAG ..." ...]
# Each lands in raytracer-challenge-rs_amd/lib_exp_NAME/librtamd.so; the
# extension picks it up through LD_LIBRARY_PATH (its RUNPATH yields to it),
# see tools/archive/exp_time.sh.
set -e
cd "$(dirname "$0")/../raytracer-challenge-rs_amd"
while [ $# -ge 2 ]; do
  name=$1 flags=$2; shift 2
  make -s -j8 LIB="lib_exp_$name" OBJ="lib_exp_$name/obj" EXTRA="$flags" "lib_exp_$name/librtamd.so"
  echo "built lib_exp_$name ($flags)"
done
