#!/bin/bash
# Build tuning variants of the device/front-end libraries into yulio-raytracer_amd/lib_variants/<name>
# usage: tools/build_variants.sh name1 "-DFLAG=1 ..." name2 "..."
set -e
cd "$(dirname "$0")/../yulio-raytracer_amd"
# the front end finds its resources at <libdir>/../resources
mkdir -p lib_variants && ln -sfn ../resources lib_variants/resources
while [ $# -ge 2 ]; do
  make -j8 BUILD=build_v/$1 LIB=lib_variants/$1 EXTRA="$2" > /dev/null
  echo "built $1: $2"
  shift 2
done
