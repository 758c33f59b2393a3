# round 6: (1) the forced-timeout KeyGen test on the default build and on a build with the host's
# flag / scratch re-zeroing removed (variants/libqrkem_nodirty.so: the test must FAIL there -- it is
# sensitive to a stale flag); (2) the single-shot service probe v2; (3) the schedule A/B (TAG=a)
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/b${TAG:-}
V=quantum-resistant-p2p_amd/qrkem/variants
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py -k forced_timeout > $O/forced_default.log 2>&1 || { tail -30 $O/forced_default.log; exit 1; }
tail -1 $O/forced_default.log
QRKEM_LIBRARY=$V/libqrkem_nodirty.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_mlkem.py -k forced_timeout > $O/forced_nodirty.log 2>&1
rc=$?
tail -1 $O/forced_nodirty.log
[ $rc -eq 1 ] || { echo "nodirty run: expected test failures (rc 1), got rc $rc"; exit 1; }
probe ss_service ss_service_probe.hip && cat $O/ss_service.txt
TAG=${TAG:-a} bash tools/r6_sched.sh
