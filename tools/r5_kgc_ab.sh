# round 5: batched KeyGen core at 4 waves per SIMD (128 VGPRs, spills) with / without the row prefetch,
# measured through the handshake driver (2 KeyGen per handshake)
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/kgc && abx 3 base=default w4=kgw4 w4np=kgw4np -- --mode handshake --steps 6 --warmup 2 --no-cpu || exit 1
echo kgc_done
