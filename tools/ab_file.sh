#!/bin/bash
# A/B build of the working tree's engine library with one source file replaced by another file:
#   tools/ab_file.sh NAME FILE REPLACEMENT  ->  ab/libfr_engine_NAME.so  (run via FR_ENGINE_LIB)
set -e
NAME=$1; FILE=$2; REPL=$3
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/abf_$NAME/pkg/csrc
rm -rf /tmp/abf_$NAME; mkdir -p /tmp/abf_$NAME/pkg; ln -s $R/include /tmp/abf_$NAME/include
cp -r $R/multi-modal-food-recommendation_amd/csrc $T; rm -rf $T/build
cp $REPL $T/$FILE
mkdir -p $R/ab
make -s -j8 -C $T OUT_DIR=$R/ab OUT=$R/ab/libfr_engine_$NAME.so
echo built $R/ab/libfr_engine_$NAME.so
