#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Compiles the reference's own callers (cpuParallel/main.cpp,
# Cipher.cpp, cloud.cpp) IN PLACE and UNCHANGED against this repo's include/ and
# libtfhe_amd.so — the drop-in proof of SURVEY.md §8(b)/(f) row 2 — plus our driver
# tests/callers/cipher_ops.cpp over the reference's Cipher class.  Only the include and
# link lines differ from cpuParallel/compile.sh:1-2.  Outputs go to oracle/_ref/callers/
# (git-ignored; travels to the GPU box with the snapshot).
set -euo pipefail
REF=${TFHE_REFERENCE:-/root/reference}/cpuParallel
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(dirname "$HERE")
OUT="$HERE/_ref/callers"
LIBDIR="$REPO/cpu-gpu-tfhe_amd/lib"
if [ ! -d "$REF" ]; then echo "reference not present at $REF; skipping callers build"; exit 0; fi
if [ ! -f "$LIBDIR/libtfhe_amd.so" ]; then echo "build libtfhe_amd.so first" >&2; exit 1; fi
mkdir -p "$OUT"
INC="-I$REPO/include -I$REPO -I$REF"
LINK="-L$LIBDIR -ltfhe_amd -Wl,-rpath,$LIBDIR"
g++ -std=c++11 -O2 $INC "$REF/main.cpp" -o "$OUT/main" $LINK -lgomp
g++ -std=c++11 -O2 -fopenmp $INC "$REF/cloud.cpp" "$REF/Cipher.cpp" -o "$OUT/cloud" $LINK
g++ -std=c++11 -O2 -fopenmp $INC "$REPO/tests/callers/cipher_ops.cpp" "$REF/Cipher.cpp" -o "$OUT/cipher_ops" $LINK
# the same with Cipher.cpp's own OpenMP loops switched on (its `#define PARALLEL`, left commented
# out at Cipher.cpp:13, given on the command line: the source stays unchanged)
g++ -std=c++11 -O2 -fopenmp -DPARALLEL $INC "$REPO/tests/callers/cipher_ops.cpp" "$REF/Cipher.cpp" -o "$OUT/cipher_ops_par" $LINK
echo "built $OUT/{main,cloud,cipher_ops,cipher_ops_par}"
