# round 6, last check of HEAD: the whole GPU suite, smoke, the default bench line, and a two-rank
# rehearsal of the multi-GPU bench path on this one GPU (gloo for the reduce, both ranks on cuda:0)
set -o pipefail
cd /root/repo && source tools/gpu.sh && out r6/last3
SUITE_TIMEOUT=1500 suite tests || exit 1
smoke || exit 1
bench bench_default && cut -c1-200 $O/bench_default.json || exit 1
QRK_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu \
  > $O/rehearsal_2ranks.json 2> $O/rehearsal_2ranks.err || exit 1
cut -c1-300 $O/rehearsal_2ranks.json
echo last_done
