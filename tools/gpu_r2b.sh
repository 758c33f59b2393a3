set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 900 bash tools/ab.sh 3 default nofence nopf4 nopf4nf -- --steps 10 --warmup 3 --streams 1 > gpurun_out/r2b/ab.jsonl 2> gpurun_out/r2b/ab.err
