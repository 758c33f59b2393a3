# round 5, second final build (direct rho at chunks <= 2^15, wire codec in-flight loads, HQC LDS
# pricing): the whole GPU suite, smoke, the default bench line, rocprofv3 trace + FETCH/WRITE + SQ
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/final2
SUITE_TIMEOUT=1500 suite tests || exit 1
smoke || exit 1
bench bench_default || exit 1
cat $O/bench_default.json
prof mlkem768 || exit 1
sq mlkem768 || exit 1
echo final2_a_done
