# round 5 final build, part A: the whole GPU suite, smoke, the default bench line
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r5/final
SUITE_TIMEOUT=1500 suite tests || exit 1
smoke || exit 1
bench bench_default || exit 1
cat $O/bench_default.json
