# Round 2 (second session) final build, part B: FrodoKEM bench lines, then the ML-KEM-768 rocprofv3
# evidence (kernel trace, FETCH_SIZE / WRITE_SIZE passes, SQ instruction-mix passes).
set -o pipefail
O=gpurun_out/final_r2b
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; }
run frodo640 --alg FrodoKEM-640-SHAKE &&
run frodo976 --alg FrodoKEM-976-SHAKE &&
run frodo1344 --alg FrodoKEM-1344-SHAKE --steps 3 --warmup 1 &&
run frodo640aes --alg FrodoKEM-640-AES &&
run frodo976aes --alg FrodoKEM-976-AES &&
run frodo1344aes --alg FrodoKEM-1344-AES --steps 3 --warmup 1 &&
run handshake_frodo976aes --alg FrodoKEM-976-AES --mode handshake --steps 3 --warmup 1 &&
bash tools/profile.sh mlkem768_r2b > $O/prof.log 2>&1 &&
bash tools/pmc_sq.sh mlkem768_r2b >> $O/prof.log 2>&1
