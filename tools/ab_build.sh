#!/bin/bash
# A/B builds of the engine library with one source file taken from another commit:
#   tools/ab_build.sh NAME COMMIT FILE[,FILE...] [extra .cpp]  ->  ab/libfr_engine_NAME.so  (run via FR_ENGINE_LIB)
set -e
NAME=$1; COMMIT=$2; FILE=$3; EXTRA=$4
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/ab_$NAME/pkg/csrc
rm -rf /tmp/ab_$NAME; mkdir -p /tmp/ab_$NAME; ln -s $R/include /tmp/ab_$NAME/include
mkdir -p /tmp/ab_$NAME/pkg; cp -r $R/multi-modal-food-recommendation_amd/csrc $T; rm -rf $T/build
for F in ${FILE//,/ }; do git -C $R show $COMMIT:multi-modal-food-recommendation_amd/csrc/$F > $T/$F; done
SRCS_CPP="fr_abi.cpp fr_io.cpp fr_comm.cpp fr_error.cpp fr_sampler.cpp"
if [ -n "$EXTRA" ]; then cp $EXTRA $T/; SRCS_CPP="$SRCS_CPP $(basename $EXTRA)"; fi
mkdir -p $R/ab
make -s -j8 -C $T OUT_DIR=$R/ab OUT=$R/ab/libfr_engine_$NAME.so SRCS_CPP="$SRCS_CPP"
echo built $R/ab/libfr_engine_$NAME.so
