# round 5, last check of HEAD: the whole GPU suite, smoke, the default bench line
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/final3
SUITE_TIMEOUT=1500 suite tests || exit 1
smoke || exit 1
bench bench_default || exit 1
echo final3_done
