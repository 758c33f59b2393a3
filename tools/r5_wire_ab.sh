# round 5, wire codec: base64 encode / decode with four chunks' loads in flight per
# lane -- wire tests, same-box A/B against the round-5 docs head (abtrees/r5head), a profiled line
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/wire
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wire.py \
  > $O/tests_wire.log 2>&1 || { tail -30 $O/tests_wire.log; exit 1; }
tail -2 $O/tests_wire.log
out r5/wire/ab && abx 3 new=default old=tree:abtrees/r5head -- --mode wire --steps 20 --warmup 3 --no-profile --no-cpu || exit 1
out r5/wire && bench wire_mlkem768 --mode wire --steps 20 --warmup 3 || exit 1
echo wire_done
