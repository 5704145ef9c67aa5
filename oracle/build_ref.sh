#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Compiles the reference's own pure-C++ leaf sources IN PLACE
# (read-only, from /root/reference/gpuParallel) plus our flat-array driver into
# oracle/_ref/libtfheref.so.  Nothing is copied into the repo; oracle/_ref/ is git-ignored.
# The rest of the reference path (FFT, bootstrapping, key switch) needs cufftXt.h /
# fftw3.h / nvcc and is unbuildable here.
set -euo pipefail
REF=${TFHE_REFERENCE:-/root/reference}/gpuParallel
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF" ]; then echo "reference not present at $REF; skipping _ref build"; exit 0; fi
mkdir -p "$OUT"
SRCS="numeric-functions multiplication lwe-functions lwesamples lwekey lweparams"
OBJS=""
for f in $SRCS; do
  g++ -std=c++11 -O2 -fPIC -fwrapv -x c++ -c "$REF/$f.cu" -I"$REF" -o "$OUT/$f.o"
  OBJS="$OBJS $OUT/$f.o"
done
g++ -std=c++11 -O2 -fPIC -fwrapv -c "$HERE/ref_driver.cpp" -I"$REF" -o "$OUT/ref_driver.o"
g++ -shared -o "$OUT/libtfheref.so" $OBJS "$OUT/ref_driver.o"
rm -f $OBJS "$OUT/ref_driver.o"
g++ -std=c++11 -Wno-invalid-offsetof -I"$REF" "$HERE/ref_layout.cpp" -o "$OUT/ref_layout"
echo "built $OUT/libtfheref.so"
