# Re-entry check: 64-bit shift probe, full GPU suite, smoke, default bench line (ML-KEM-768 2^20).
set -o pipefail
O=gpurun_out/check
mkdir -p $O
timeout -k 10 120 tools/rot64_probe > $O/rot64_probe.json 2> $O/rot64_probe.err &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/t.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
