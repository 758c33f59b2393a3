set -o pipefail
mkdir -p gpurun_out/r2m
for u in 1 2 4 24; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -DQRK_COOP_UNROLL=$u -o /tmp/kcp$u tools/keccak_coop_probe.hip || exit 1
done
for u in 1 2 4 24; do
  echo "unroll $u $(timeout -k 5 60 /tmp/kcp$u)" >> gpurun_out/r2m/coop_unroll.txt || exit 1
done
