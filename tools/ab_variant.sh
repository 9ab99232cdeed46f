#!/bin/bash
# A/B build of the working tree's engine library with one source file edited by a sed expression:
#   tools/ab_variant.sh NAME FILE 'sed-expr'  ->  ab/libfr_engine_NAME.so  (run via FR_ENGINE_LIB)
set -e
NAME=$1; FILE=$2; EXPR=$3
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/abv_$NAME/pkg/csrc
rm -rf /tmp/abv_$NAME; mkdir -p /tmp/abv_$NAME/pkg; ln -s $R/include /tmp/abv_$NAME/include
cp -r $R/multi-modal-food-recommendation_amd/csrc $T; rm -rf $T/build
sed -i "$EXPR" $T/$FILE
mkdir -p $R/ab
make -s -j8 -C $T OUT_DIR=$R/ab OUT=$R/ab/libfr_engine_$NAME.so
echo built $R/ab/libfr_engine_$NAME.so
