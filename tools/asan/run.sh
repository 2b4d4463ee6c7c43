#!/bin/bash
# AddressSanitizer build of libdfk's HOST code (device code unchanged; -fsanitize only on the host side of each
# hipcc compile) plus tools/asan/host_check.cpp, run on the CPU (no GPU needed: nothing is launched).
#   bash tools/asan/run.sh [outdir]      (default /tmp/dfk_asan)
set -e -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${1:-/tmp/dfk_asan}
mkdir -p $OUT
HIPCC=/opt/rocm/bin/hipcc
FL="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
objs=""
for f in $R/deepfake_amd/csrc/*.hip; do
  o=$OUT/$(basename $f .hip).o
  $HIPCC $FL -c $f -o $o
  objs="$objs $o"
done
$HIPCC -O1 -g -std=c++17 -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -c \
    $R/tools/asan/host_check.cpp -o $OUT/host_check.o
$HIPCC --offload-arch=gfx950 -fsanitize=address -o $OUT/host_check $OUT/host_check.o $objs
ASAN_OPTIONS=detect_leaks=0 $OUT/host_check
