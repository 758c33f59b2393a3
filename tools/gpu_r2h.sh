set -o pipefail
mkdir -p gpurun_out/r2h
for c in 1048576 262144 65536 32768 16384; do
  timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu --chunk $c --streams 1 > gpurun_out/r2h/chunk_$c.json 2> gpurun_out/r2h/chunk_$c.err || exit 1
done
