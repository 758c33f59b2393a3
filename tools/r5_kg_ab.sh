# round 5: single-shot KeyGen -- pipelined (default) vs round-4 multi-workgroup kernel, interleaved,
# plus the pipelined kernel's phase trace and the ML-KEM GPU tests on the default build
set -o pipefail
cd /root/repo && O=gpurun_out/r5/kg${TAG:-} && mkdir -p $O
V=quantum-resistant-p2p_amd/qrkem/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mlkem.py tests/test_gpu_ordering.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
QRKEM_LIBRARY=$V/libqrkem_sstrace.so timeout -k 10 120 python -u tools/single_shot_trace.py > $O/trace_pipe.json || exit $?
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "pipe", /' >> $O/ab_pipe_vs_multi.jsonl || exit $?
  QRKEM_LIBRARY=$V/libqrkem_kgmulti.so timeout -k 10 120 python -u tools/single_shot_breakdown.py ML-KEM-768 | sed 's/^{/{"variant": "multi", /' >> $O/ab_pipe_vs_multi.jsonl || exit $?
done
cat $O/trace_pipe.json $O/ab_pipe_vs_multi.jsonl
