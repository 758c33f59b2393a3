# round 6: the forced-timeout test with the flag-residue check, on the default build (must pass) and
# on a build without the host's re-zeroing (nodirty: every case must fail now, not only a racy one)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r6/forced2 && O=gpurun_out/r6/forced2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py -k forced_timeout > $O/forced_default.log 2>&1 || { tail -30 $O/forced_default.log; exit 1; }
tail -1 $O/forced_default.log
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_nodirty.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py -k forced_timeout > $O/forced_nodirty.log 2>&1
tail -1 $O/forced_nodirty.log
grep -c PASSED $O/forced_nodirty.log || true
