#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Compiles the reference's own pure-C++ leaf sources IN PLACE
# (read-only, from /root/reference/gpuParallel) plus our flat-array driver into
# oracle/_ref/libtfheref.so.  Nothing is copied into the repo; oracle/_ref/ is git-ignored.
# tgsw.cu (TGswParams: h[], offset), tlwe.cu (TLweParams) and lwekeyswitch.cu (the ks[i][j][h]
# index map) pin the decomposition constants and the key-switching key layout.  The rest of the
# reference path (FFT, bootstrapping, decomposition, key switch) needs cufftXt.h / fftw3.h /
# nvcc and is unbuildable here.
set -euo pipefail
REF=${TFHE_REFERENCE:-/root/reference}/gpuParallel
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF" ]; then echo "reference not present at $REF; skipping _ref build"; exit 0; fi
mkdir -p "$OUT"
SRCS="numeric-functions multiplication lwe-functions lwesamples lwekey lweparams"
# only their parameter / index constructors are used; the rest of tlwe.cu references the
# CUDA-only polynomial allocators, so these are built hidden and garbage-collected per function
PARAM_SRCS="tgsw tlwe lwekeyswitch"
OBJS=""
for f in $SRCS; do
  g++ -std=c++11 -O2 -fPIC -fwrapv -x c++ -c "$REF/$f.cu" -I"$REF" -o "$OUT/$f.o"
  OBJS="$OBJS $OUT/$f.o"
done
for f in $PARAM_SRCS; do
  g++ -std=c++11 -O2 -fPIC -fwrapv -fvisibility=hidden -ffunction-sections -fdata-sections -x c++ -c "$REF/$f.cu" -I"$REF" -o "$OUT/$f.o"
  OBJS="$OBJS $OUT/$f.o"
done
g++ -std=c++11 -O2 -fPIC -fwrapv -c "$HERE/ref_driver.cpp" -I"$REF" -o "$OUT/ref_driver.o"
g++ -shared -Wl,--gc-sections -o "$OUT/libtfheref.so" $OBJS "$OUT/ref_driver.o"
rm -f $OBJS "$OUT/ref_driver.o"
g++ -std=c++11 -Wno-invalid-offsetof -I"$REF" "$HERE/ref_layout.cpp" -o "$OUT/ref_layout"
echo "built $OUT/libtfheref.so"
