# round 6: the fix-up counters after a chunk that fails after the parity flip -- the new
# test on the default build (must pass) and on a build without the fixc_dirty re-zero (must fail)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r6/fixc && O=gpurun_out/r6/fixc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py -k "rezeroed_after_failed_chunk or fixup_counters_across_calls" > $O/default.log 2>&1 || { tail -30 $O/default.log; exit 1; }
tail -1 $O/default.log
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_nofixdirty.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py -k rezeroed_after_failed_chunk > $O/without_rezero.log 2>&1
tail -1 $O/without_rezero.log
grep -E "^E .*assert sorted" $O/without_rezero.log | head -2 || true
