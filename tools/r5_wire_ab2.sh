# round 5, wire codec: chunks in flight per lane, 2 / 4 (default) / 8
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/wire/ab2 && abx 3 u4=default u2=u2 u8=u8 -- --mode wire --steps 20 --warmup 3 --no-cpu || exit 1
echo wire2_done
