#!/bin/bash
# A/B build of libmmf_hip.so into variants/<name>/ with extra compile flags, reusing the in-tree
# objects of every file but the ones listed in FILES (default effnet.hip):
#   bash tools/build_variant.sh <name> "<-D flags>" [src_dir]
# src_dir defaults to the in-tree csrc (pass an extracted older tree for a baseline build).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2
SRC=${3:-$R/multi-modal-misinformation-detection-with-explanation-generation_amd/csrc}
FILES=${FILES:-effnet.hip}
BD=$SRC/build_$NAME
mkdir -p $BD
cp -p $R/multi-modal-misinformation-detection-with-explanation-generation_amd/csrc/build/*.o $BD/ 2>/dev/null || true
for f in $FILES; do rm -f $BD/${f%.*}.o; done
touch $BD/*.o
for f in $FILES; do touch $SRC/$f; done
make -s -C $SRC -j8 BUILD=build_$NAME LIB=$R/variants/$NAME/libmmf_hip.so EXTRA="$FLAGS"
echo "variants/$NAME/libmmf_hip.so"
