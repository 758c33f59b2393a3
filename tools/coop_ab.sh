# A/B of the wave-cooperative Keccak variants (tools/keccak_coop_probe.hip): correctness against
# the lane-per-state permutation and single-wave cycles per permutation.
set -o pipefail
mkdir -p gpurun_out/coop
for v in "v2 -DQRK_COOP_V1=0" "v2chi -DQRK_COOP_V1=0 -DQRK_COOP_CHI_DPP=1" "v1 -DQRK_COOP_V1=1"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w $2 $3 -o /tmp/kcp_$1 tools/keccak_coop_probe.hip || exit 1
  echo "$1 $(timeout -k 5 60 /tmp/kcp_$1)" >> gpurun_out/coop/ab2.txt || exit 1
done
