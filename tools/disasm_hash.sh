#!/bin/bash
# Hash of the default build's device code: every csrc/*.hip compiled device-only for gfx950 with
# the Makefile's flags, disassembled (llvm-objdump -d, instructions only), one SHA-256 per file
# plus one over all of them.  Used to show a source clean-up leaves the shipped kernels unchanged:
#   tools/disasm_hash.sh [extra hipcc flags]   -> prints "<sha256>  <file>" lines and "<sha256>  ALL"
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
C=${CSRC:-$R/quantum-resistant-p2p_amd/csrc}
T=$(mktemp -d /tmp/dhash.XXXX)
for f in $(cd "$C" && ls *.hip); do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -w --cuda-device-only "$@" -c "$C/$f" -o "$T/${f%.hip}.bundle" &&
    /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
      --input="$T/${f%.hip}.bundle" --output="$T/${f%.hip}.co" &
done
wait
for f in $(cd "$T" && ls *.co); do
  /opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn --no-leading-addr "$T/$f" | grep -v 'file format' > "$T/${f%.co}.s"
  echo "$(sha256sum < "$T/${f%.co}.s" | cut -c1-64)  $f"
done
echo "$(cat "$T"/*.s | sha256sum | cut -c1-64)  ALL"
rm -rf "$T"
