# round 5: staged record absorbs for the ML-KEM Encaps front and J -- parity,
# interleaved A/B at 2^20 and 2^16, then a FETCH_SIZE pass of each build
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/stage
SUITE_TIMEOUT=1200 suite tests/test_gpu_mlkem.py tests/test_gpu_fullsize.py tests/test_gpu_schedule.py || exit 1
out r5/stage/b20 && abx 4 stage=default nostage=nostage -- --steps 20 --warmup 5 --no-profile || exit 1
out r5/stage/b16 && abx 3 stage=default nostage=nostage -- --log2-batch 16 --steps 30 --warmup 5 --no-profile || exit 1
out r5/stage/fetch
for t in default nostage; do
  L=$R/quantum-resistant-p2p_amd/qrkem/libqrkem.so; [ $t != default ] && L=$R/quantum-resistant-p2p_amd/qrkem/variants/libqrkem_$t.so
  ( export TMPDIR=/tmp QRKEM_LIBRARY=$L; cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/$t" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile > "$O/$t.json" 2> "$O/$t.err" ) || exit 1
done
echo stage_done
