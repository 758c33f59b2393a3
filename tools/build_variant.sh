#!/bin/bash
# Build an experimental libqrkem variant with extra -D flags (kernel tuning sweeps):
#   [CSRC=<other csrc dir>] tools/build_variant.sh <tag> -DQRK_SMALL_MAX=512 ...
# Output: quantum-resistant-p2p_amd/qrkem/variants/libqrkem_<tag>.so (git-ignored; load it
# with QRKEM_LIBRARY=<path>).  The default build is untouched.
set -euo pipefail
tag=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=${CSRC:-$R/quantum-resistant-p2p_amd/csrc}
O=$R/build/variant_$tag
mkdir -p "$O" "$R/quantum-resistant-p2p_amd/qrkem/variants"
for f in $(cd "$C" && ls *.hip | sed "s/\.hip$//"); do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c "$C/$f.hip" -o "$O/$f.o" &
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -fPIC -std=c++17 "$@" -c "$C/abi.cpp" -o "$O/abi.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/quantum-resistant-p2p_amd/qrkem/variants/libqrkem_$tag.so" "$O"/*.o
echo "built variants/libqrkem_$tag.so"
