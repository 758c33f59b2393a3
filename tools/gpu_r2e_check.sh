# Last check of the committed build: full GPU suite and smoke into gpurun_out/final_r2e/.
set -o pipefail
O=gpurun_out/final_r2e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/mlkem768.json 2> $O/mlkem768.err
